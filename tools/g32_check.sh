# Group-32 (GGUF Q4_0 / Q8_0) weights: kernel and engine parity, plus regression of the G128 kernels
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_g32.py tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g32_tests.log 2>&1
