#!/bin/bash
# Persistent decode diagnosis: fill traces and the 7B bench line (TI_PDS=1) for the exp builds
#   pft     product + trace          pring   the ring alone (consumers acquire / release only)
#   pringl2 the ring alone, every piece from L2     pprio  loader at s_setprio 3     pdef  no nt
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r4d_bench.txt
for v in pring pringl2 pft pprio pdef; do
  L=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so
  DETAIL=0 TI_LIB=$L timeout -k 10 200 python3 -u tools/pds_ftrace.py > gpurun_out/r4d_ftrace_$v.txt 2>&1 || exit 1
  TI_PDS=1 TI_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 50 --warmup 8 --no-cpu-baseline > gpurun_out/r4d_$v.json 2>> gpurun_out/r4d_bench.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/r4d_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'))")" >> gpurun_out/r4d_bench.txt
done
echo "diag done"
