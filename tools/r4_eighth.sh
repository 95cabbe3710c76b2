#!/bin/bash
# Persistent decode, consumers with interleaved MFMA chains: bit-identity tests, the fill trace (exp/pl4),
# phase timeline, 7B persistent vs graph, TinyLlama persistent vs graph.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4h_pds_tests.txt 2>&1 || exit 1
echo "pds tests ok"
DETAIL=1 TI_LIB=$GRAFT_REPO_ROOT/exp/pl4/libturboinfer_amd.so timeout -k 10 200 python3 -u tools/pds_ftrace.py > gpurun_out/r4h_ftrace.txt 2>&1 || exit 1
TI_PDS=1 TI_PDS_TS=1 timeout -k 10 200 python3 -u tools/pds_phases.py > gpurun_out/r4h_phases.txt 2>&1 || exit 1
: > gpurun_out/r4h_bench.txt
for v in pds graph tlpds tlgraph; do
  P=0; M=llama2-7b
  case $v in pds) P=1;; tlgraph) M=tinyllama-1.1b;; tlpds) P=1; M=tinyllama-1.1b;; esac
  TI_PDS=$P timeout -k 10 200 python3 -u bench.py --model $M --steps 100 --warmup 8 --no-cpu-baseline > gpurun_out/r4h_$v.json 2>> gpurun_out/r4h_bench.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/r4h_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'))")" >> gpurun_out/r4h_bench.txt
done
echo "done8"
