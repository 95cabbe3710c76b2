# A/B of the ring-issue delay knob (TI_GEMV_RING_DELAY builds in turboinfer_amd/lib/exp/)
set -e
for i in 1 2; do
  for v in d0 d10 d25 d60; do
    lib=turboinfer_amd/lib/exp/lib_$v.so; [ $v = d0 ] && lib=turboinfer_amd/lib/libturboinfer_amd.so
    TI_LIB=$lib timeout -k 10 200 python bench.py --steps 512 --no-cpu-baseline --kernel-reps 200 > gpurun_out/ab_${v}_$i.log 2>&1
  done
done
