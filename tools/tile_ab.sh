# Prefill tile GEMM: 64-column workgroups for narrow shapes (TI_TILE_NARROW) A/B, parity, timing
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill.py tests/test_gpu_batched.py -x -q --timeout 120 --timeout-method thread > gpurun_out/prefill_tests.log 2>&1
TI_TILE_NARROW=1 timeout -k 10 200 python3 tools/rows_bench.py 256 > gpurun_out/tile_narrow1.txt 2>&1
TI_TILE_NARROW=0 timeout -k 10 200 python3 tools/rows_bench.py 256 > gpurun_out/tile_narrow0.txt 2>&1
timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/prefill.txt 2>&1
