# Prefill attention: K/V ring depth A/B (TI_PF_RING builds under exp/, default lib = 4)
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in r2 r3; do
  TI_LIB=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill_attn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pfr_$v.log 2>&1
  TI_LIB=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so timeout -k 10 120 python3 -u tools/prefill_attn_time.py > gpurun_out/pfr_time_$v.txt 2>&1
done
timeout -k 10 120 python3 -u tools/prefill_attn_time.py > gpurun_out/pfr_time_r4.txt 2>&1
