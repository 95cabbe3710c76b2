# Group-32 (GGUF Q4_0 / Q8_0) weights: kernel, engine and C++ API parity
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_g32.py tests/test_cpp_api.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g32_tests.log 2>&1
