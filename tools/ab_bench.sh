mkdir -p gpurun_out/ab
run() { # name lib extra-args
  local n=$1 l=$2; shift 2
  if [ "$l" = base ]; then unset TI_LIB; else export TI_LIB=turboinfer_amd/lib/exp/lib_$l.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --kernel-reps 20 "$@" > gpurun_out/ab/$n.log 2>&1 || return 1
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(sys.argv[2], d['value'], {k:v['avg_us'] for k,v in d['kernels'].items()}, flush=True)" gpurun_out/ab/$n.log $n
}
