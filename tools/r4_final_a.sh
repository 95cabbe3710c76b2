#!/bin/bash
# Round-4 end (a): the whole GPU suite with the deep-parity error log, then the side-config bench lines.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/r4_deep_parity.jsonl
TI_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/r4_deep_parity.jsonl timeout -k 10 700 python3 -u -m pytest tests/ -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4_gpu_suite.txt 2>&1
echo "suite rc=$?"
bash tools/side_configs.sh r4 || exit 1
echo "side done"
