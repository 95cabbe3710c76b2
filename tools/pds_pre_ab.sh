#!/bin/bash
# Persistent decode: ring units issued before a hand-off (TI_PDS_PRE 0/2/4/8) A/B, bench + timeline.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pds_tests.log 2>&1
: > gpurun_out/pds_pre_ab.txt
for v in 2 0 4 8 graph; do
  if [ $v = graph ]; then L=""; P=0; elif [ $v = 2 ]; then L=""; P=1; else L=$GRAFT_REPO_ROOT/exp/pre$v/libturboinfer_amd.so; P=1; fi
  TI_LIB=$L TI_PDS=$P timeout -k 10 200 python3 bench.py --steps 256 --no-cpu-baseline > gpurun_out/pds_pre_$v.json 2>> gpurun_out/pds_pre_ab.err
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/pds_pre_$v.json'));print(d['value'], d['ms_per_step'])")" >> gpurun_out/pds_pre_ab.txt
done
timeout -k 10 150 python3 tools/pds_phases.py > gpurun_out/pds_pre2_phases.txt 2>&1
