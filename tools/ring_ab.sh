#!/bin/bash
# RECORD ONLY: TI_GEMV_WG_PER_CU is no longer read by the library (DESIGN 4.1 (a second workgroup per CU measured slower)); the script stops here.
echo "TI_GEMV_WG_PER_CU is gone (DESIGN 4.1 (a second workgroup per CU measured slower))"; exit 2
# Fused-GEMV ring depth (TI_GEMV_RING_VGPRS 20 = product, exp/r24, exp/r32 builds) and two
# workgroups per CU (TI_GEMV_WG_PER_CU=2) on the one-stream 7B and TinyLlama benches.
# Variant builds: make BUILD=/tmp/build_rNN LIB=exp/rNN/libturboinfer_amd.so EXTRA=-DTI_GEMV_RING_VGPRS=NN
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ring
run() { # name model env...
  local n=$1 m=$2; shift 2
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu-baseline --kernel-reps 20 --steps 200 --model $m > gpurun_out/ring/$n.log 2>&1
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(sys.argv[2], d['value'], {k:v['avg_us'] for k,v in d.get('kernels',{}).items()}, flush=True)" gpurun_out/ring/$n.log $n
}
X=$GRAFT_REPO_ROOT/exp
for i in 1 2; do
  run tl_r20_$i tinyllama-1.1b
  run tl_r24_$i tinyllama-1.1b TI_LIB=$X/r24/libturboinfer_amd.so
  run tl_r32_$i tinyllama-1.1b TI_LIB=$X/r32/libturboinfer_amd.so
  run tl_r20_wg2_$i tinyllama-1.1b TI_GEMV_WG_PER_CU=2
  run tl_r32_wg2_$i tinyllama-1.1b TI_LIB=$X/r32/libturboinfer_amd.so TI_GEMV_WG_PER_CU=2
done
for i in 1 2; do
  run 7b_r20_$i llama2-7b
  run 7b_r24_$i llama2-7b TI_LIB=$X/r24/libturboinfer_amd.so
  run 7b_r32_$i llama2-7b TI_LIB=$X/r32/libturboinfer_amd.so
done
