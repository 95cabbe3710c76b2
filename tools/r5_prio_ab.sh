#!/bin/bash
# RECORD ONLY: TI_GEMV_PRIO lost this A/B (profiles/r5_gemv_prio_ab.txt) and its code was removed afterwards, so on
# this tree both arms would be the same build; the script stops here.
echo "TI_GEMV_PRIO was removed after this A/B (profiles/r5_gemv_prio_ab.txt)"; exit 2
# A/B: static s_setprio in gemv_wq_kernel (TI_GEMV_PRIO 0 / 1 / 2, builds tools/bin/p<N>):
# per-launch phase probes, then the default bench interleaved 3x per arm.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/prio
mkdir -p $O
for p in "" p1 p2; do
  timeout -k 10 120 tools/bin/probe_gemv_e4$p 64 > $O/probe_e4$p.txt 2>&1 || exit 1
done
for r in 1 2 3; do
  for p in p0 p1 p2; do
    L=""; [ $p = p0 ] || L=$GRAFT_REPO_ROOT/tools/bin/$p/libturboinfer_amd.so
    TI_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --kernel-reps 20 > $O/bench_${p}_$r.json 2>$O/bench_${p}_$r.err || exit 1
    python3 -c "import json;d=json.load(open('$O/bench_${p}_$r.json'));print('$p',$r,d['value'],{k:v['avg_us'] for k,v in d['kernels'].items()})"
  done
done
