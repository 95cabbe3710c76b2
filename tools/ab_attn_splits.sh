# A/B: single-stream attention over 16 splits (2 workgroups per CU) merged by the O projection
# (TI_ATTN_MAX_PART_SPLITS=16 build in turboinfer_amd/lib/exp/) vs the default 8
set -e
L16=turboinfer_amd/lib/exp/lib_ps16.so
TI_LIB=$L16 TI_ATTN_TARGET=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py -x -q --timeout 120 --timeout-method thread -k engine > gpurun_out/ab_sp_test.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 512 --no-cpu-baseline > gpurun_out/ab_sp8_$i.log 2>&1
  TI_LIB=$L16 TI_ATTN_TARGET=512 timeout -k 10 200 python bench.py --steps 512 --no-cpu-baseline > gpurun_out/ab_sp16_$i.log 2>&1
  TI_LIB=$L16 timeout -k 10 200 python bench.py --steps 512 --no-cpu-baseline > gpurun_out/ab_sp8b_$i.log 2>&1
done
