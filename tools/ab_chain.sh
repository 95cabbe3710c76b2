# A/B of chained vs graph decode steps (GPU box): bench lines into gpurun_out/ab/
mkdir -p gpurun_out/ab
run() { # name lib chain
  local n=$1 l=$2 c=$3
  if [ "$l" = base ]; then unset TI_LIB; else export TI_LIB=turboinfer_amd/lib/exp/lib_$l.so; fi
  TI_CHAIN=$c timeout -k 10 200 python bench.py --no-cpu-baseline --kernel-reps 5 > gpurun_out/ab/$n.log 2>&1 || return 1
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(sys.argv[2], d['value'], d['ms_per_step'], flush=True)" gpurun_out/ab/$n.log $n
}
