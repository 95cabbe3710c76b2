# Prefill tile GEMM (3-stage LDS-DMA pipeline): parity, per-shape timing, prefill; sampler tests
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py tests/test_gpu_batched.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tile_tests.log 2>&1
TI_ATTN_PREFILL=0 timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/prefill_old_attn.txt 2>&1
timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/prefill.txt 2>&1
