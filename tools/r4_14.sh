#!/bin/bash
# Persistent decode with the scale loads sharing the gathers' round trip: bit-identity tests, the phase
# timeline, 7B persistent vs graph.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4n_pds_tests.txt 2>&1 || exit 1
echo "pds tests ok"
TI_PDS=1 TI_PDS_TS=1 timeout -k 10 200 python3 -u tools/pds_phases.py > gpurun_out/r4n_phases.txt 2>&1 || exit 1
: > gpurun_out/r4n_bench.txt
for v in pds graph; do
  P=0; [ $v = pds ] && P=1
  TI_PDS=$P timeout -k 10 200 python3 -u bench.py --steps 100 --warmup 8 --no-cpu-baseline > gpurun_out/r4n_$v.json 2>> gpurun_out/r4n_bench.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/r4n_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'))")" >> gpurun_out/r4n_bench.txt
done
echo "done14"
