#!/bin/bash
# Second round-4 GPU call: the persistent launch's per-fill ring trace (exp/pft, -DTI_PDS_FTRACE=1),
# the re-run of the two suite failures after their fixes, TinyLlama (configs[1]) graph vs
# persistent, then the round-head interleave.  Stops at the first failure.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TI_LIB=$GRAFT_REPO_ROOT/exp/pft/libturboinfer_amd.so timeout -k 10 200 python3 -u tools/pds_ftrace.py > gpurun_out/r4_ftrace.txt 2>&1 || exit 1
echo "ftrace done"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_batched.py tests/test_cpp_api.py -x -q -m gpu -k "fold or contract" --timeout 120 --timeout-method thread > gpurun_out/r4_refix.txt 2>&1
echo "refix rc=$?"
: > gpurun_out/r4_tl.txt
for v in graph pds; do
  P=0; [ $v = pds ] && P=1
  TI_PDS=$P timeout -k 10 200 python3 -u bench.py --model tinyllama-1.1b --steps 200 --warmup 16 --no-cpu-baseline > gpurun_out/tl_$v.json 2>> gpurun_out/r4_tl.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/tl_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('pds'))")" >> gpurun_out/r4_tl.txt
done
echo "tinyllama done"
bash tools/r4_heads_ab.sh || exit 1
echo "heads done"
