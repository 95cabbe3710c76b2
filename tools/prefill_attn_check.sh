set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill_attn.py tests/test_gpu_prefill.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pa_tests.log 2>&1
timeout -k 10 120 python3 -u tools/prefill_attn_time.py > gpurun_out/prefill_attn_time.txt 2>&1
timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/prefill.txt 2>&1
