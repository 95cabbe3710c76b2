#!/bin/bash
# Persistent decode: fill traces with the consumers' math-done event, product vs no-GEMV-math diagnostic.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r4i_bench.txt
for v in pl4 pl4nm; do
  L=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so
  DETAIL=1 TI_LIB=$L timeout -k 10 200 python3 -u tools/pds_ftrace.py > gpurun_out/r4i_ftrace_$v.txt 2>&1 || exit 1
  TI_PDS=1 TI_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 50 --warmup 8 --no-cpu-baseline > gpurun_out/r4i_$v.json 2>> gpurun_out/r4i_bench.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/r4i_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'))")" >> gpurun_out/r4i_bench.txt
done
echo "done9"
