# A/B of the attention K/V ring depth (TI_ATTN_RING builds in turboinfer_amd/lib/exp/)
set -e
for i in 1 2; do
  for v in r2 ar3 ar4; do
    lib=turboinfer_amd/lib/exp/lib_$v.so; [ $v = r2 ] && lib=turboinfer_amd/lib/libturboinfer_amd.so
    TI_LIB=$lib timeout -k 10 200 python bench.py --steps 512 --no-cpu-baseline --kernel-reps 200 > gpurun_out/ab_${v}_$i.log 2>&1
  done
done
