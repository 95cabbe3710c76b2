#!/bin/bash
# Round-4 close: the whole GPU suite (deep-parity error log), smoke(), then the bench lines of
# configs[2] (default, with the CPU baseline) and the side configs [1], [3], [4] on one box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/r4c_deep_parity.jsonl
TI_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/r4c_deep_parity.jsonl timeout -k 10 800 python3 -u -m pytest tests/ -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4c_gpu_suite.txt 2>&1 || exit 1
echo "suite ok"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4c_smoke.txt 2>&1 || exit 1
echo "smoke ok"
timeout -k 10 300 python3 bench.py > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err || exit 1
echo "bench ok"
bash tools/side_configs.sh r4c || exit 1
echo "side done"
