set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TI_LIB=$GRAFT_REPO_ROOT/exp/xreg/libturboinfer_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_batched.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xr_tests.log 2>&1
TI_LIB=$GRAFT_REPO_ROOT/exp/xreg/libturboinfer_amd.so timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > gpurun_out/xr_rows.txt 2>&1
timeout -k 10 200 python3 tools/rows_bench.py 256 512 1024 > gpurun_out/dma_rows.txt 2>&1
TI_LIB=$GRAFT_REPO_ROOT/exp/xreg/libturboinfer_amd.so timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/xr_prefill.txt 2>&1
