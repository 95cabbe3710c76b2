#!/bin/bash
# RECORD ONLY: the balanced partition lost this A/B (profiles/r5_gemv_balance_ab.txt) and was reverted, so on
# this tree TI_GEMV_BAL does nothing; the script stops here.
echo "TI_GEMV_BAL was reverted after this A/B (profiles/r5_gemv_balance_ab.txt)"; exit 2
# Balanced partition of the fused GEMV (TI_GEMV_BAL, gemv_wq_kernel bit 24): parity tests, then
# the default bench interleaved 3x per arm (TI_GEMV_BAL=0: the plain tile split).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/bal
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_batched.py -k "balanced or splitk" tests/test_gpu_kernels.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2 3; do
  for b in 0 1; do
    TI_GEMV_BAL=$b timeout -k 10 200 python3 bench.py --no-cpu-baseline --kernel-reps 20 > $O/bench_${b}_$r.json 2>$O/bench_${b}_$r.err || exit 1
    python3 -c "import json;d=json.load(open('$O/bench_${b}_$r.json'));print('bal=$b',$r,d['value'],{k:v['avg_us'] for k,v in d['kernels'].items()})"
  done
done
