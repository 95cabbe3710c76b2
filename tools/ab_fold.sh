set -e
for i in 1 2 3; do
  TI_LIB=turboinfer_amd/lib/exp/lib_base.so timeout -k 10 200 python bench.py --steps 512 --no-cpu-baseline --kernel-reps 200 > gpurun_out/ab_base_$i.log 2>&1
  timeout -k 10 200 python bench.py --steps 512 --no-cpu-baseline --kernel-reps 200 > gpurun_out/ab_fold_$i.log 2>&1
  TI_FOLD=0 timeout -k 10 200 python bench.py --steps 512 --no-cpu-baseline --kernel-reps 200 > gpurun_out/ab_nofold_$i.log 2>&1
done
