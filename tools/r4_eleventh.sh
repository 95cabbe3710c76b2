#!/bin/bash
# Persistent decode with 8 consumer waves (each one virtual wave): bit-identity tests of that build
# (TI_LIB), then traces and the 7B / TinyLlama bench lines for 4 vs 8 consumers.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TI_LIB=$GRAFT_REPO_ROOT/exp/pc8/libturboinfer_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4k_pds_tests_c8.txt 2>&1 || exit 1
echo "pds c8 tests ok"
: > gpurun_out/r4k_bench.txt
for v in pc8 pc8l2 pl4; do
  L=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so
  DETAIL=0 TI_LIB=$L timeout -k 10 200 python3 -u tools/pds_ftrace.py > gpurun_out/r4k_ftrace_$v.txt 2>&1 || exit 1
  for M in llama2-7b tinyllama-1.1b; do
    TI_PDS=1 TI_LIB=$L timeout -k 10 200 python3 -u bench.py --model $M --steps 60 --warmup 8 --no-cpu-baseline > gpurun_out/r4k_${v}_$M.json 2>> gpurun_out/r4k_bench.err || exit 1
    echo "$v $M $(python3 -c "import json;d=json.load(open('gpurun_out/r4k_${v}_$M.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'))")" >> gpurun_out/r4k_bench.txt
  done
done
TI_PDS=1 TI_PDS_TS=1 TI_LIB=$GRAFT_REPO_ROOT/exp/pc8/libturboinfer_amd.so timeout -k 10 200 python3 -u tools/pds_phases.py > gpurun_out/r4k_phases_c8.txt 2>&1 || exit 1
echo "done11"
