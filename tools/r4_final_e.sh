#!/bin/bash
# Round-4 last check: the whole GPU suite and smoke() on the final build, then the default bench line.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/r4e_deep_parity.jsonl
TI_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/r4e_deep_parity.jsonl timeout -k 10 800 python3 -u -m pytest tests/ -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4e_gpu_suite.txt 2>&1 || exit 1
echo "suite ok"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4e_smoke.txt 2>&1 || exit 1
echo "smoke ok"
timeout -k 10 300 python3 bench.py > gpurun_out/r4e_bench.json 2> gpurun_out/r4e_bench.err || exit 1
echo "bench ok"
timeout -k 10 200 python3 tools/prefill_bench.py 512 > gpurun_out/r4e_prefill.txt 2>&1 || exit 1
echo "prefill ok"
