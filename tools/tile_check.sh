# Prefill tile GEMM: parity, per-shape timing (64-row shapes on / off), prefill
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_batched.py tests/test_gpu_prefill.py tests/test_gpu_g32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tile_tests.log 2>&1
TI_TILE_WMR1=0 timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > gpurun_out/tile_rows_w2.txt 2>&1
timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > gpurun_out/tile_rows.txt 2>&1
TI_TILE_WMR1=0 timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/prefill_w2.txt 2>&1
timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/prefill.txt 2>&1
