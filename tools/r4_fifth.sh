#!/bin/bash
# Persistent decode with 1 / 2 / 4 loader waves (and 4 with 4 fills ahead): bit-identity tests of the
# product build (4 loaders), then per variant the fill trace and the 7B bench line (TI_PDS=1).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 exp/probe_ldsdma > gpurun_out/r4e_probe_ldsdma.txt 2>&1 || exit 1
echo "probe ok"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4e_pds_tests.txt 2>&1 || exit 1
echo "pds tests ok"
: > gpurun_out/r4e_bench.txt
for v in pl4 pl2 pl1 pl4a4; do
  L=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so
  DETAIL=0 TI_LIB=$L timeout -k 10 200 python3 -u tools/pds_ftrace.py > gpurun_out/r4e_ftrace_$v.txt 2>&1 || exit 1
  TI_PDS=1 TI_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 100 --warmup 8 --no-cpu-baseline > gpurun_out/r4e_$v.json 2>> gpurun_out/r4e_bench.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/r4e_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'))")" >> gpurun_out/r4e_bench.txt
done
TI_PDS=1 TI_PDS_TS=1 timeout -k 10 200 python3 -u tools/pds_phases.py > gpurun_out/r4e_phases.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u bench.py --steps 100 --warmup 8 --no-cpu-baseline > gpurun_out/r4e_graph.json 2>> gpurun_out/r4e_bench.err || exit 1
echo "graph $(python3 -c "import json;d=json.load(open('gpurun_out/r4e_graph.json'));print(d['value'], d['ms_per_step'])")" >> gpurun_out/r4e_bench.txt
echo "done5"
