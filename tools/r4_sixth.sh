#!/bin/bash
# Persistent decode with the layer table read by scalar loads: bit-identity tests, then per loader
# count (exp builds with the fill trace) the trace and the 7B bench line, the phase timeline, the
# graph line, TinyLlama persistent vs graph.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4f_pds_tests.txt 2>&1 || exit 1
echo "pds tests ok"
: > gpurun_out/r4f_bench.txt
for v in pl4 pl2 pl1; do
  L=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so
  DETAIL=0 TI_LIB=$L timeout -k 10 200 python3 -u tools/pds_ftrace.py > gpurun_out/r4f_ftrace_$v.txt 2>&1 || exit 1
  TI_PDS=1 TI_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 100 --warmup 8 --no-cpu-baseline > gpurun_out/r4f_$v.json 2>> gpurun_out/r4f_bench.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/r4f_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'))")" >> gpurun_out/r4f_bench.txt
done
TI_PDS=1 TI_PDS_TS=1 timeout -k 10 200 python3 -u tools/pds_phases.py > gpurun_out/r4f_phases.txt 2>&1 || exit 1
for v in graph tlgraph tlpds; do
  P=0; M=llama2-7b
  case $v in tlgraph) M=tinyllama-1.1b;; tlpds) P=1; M=tinyllama-1.1b;; esac
  TI_PDS=$P timeout -k 10 200 python3 -u bench.py --model $M --steps 100 --warmup 8 --no-cpu-baseline > gpurun_out/r4f_$v.json 2>> gpurun_out/r4f_bench.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/r4f_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'))")" >> gpurun_out/r4f_bench.txt
done
echo "done6"
