#!/bin/bash
# A/B (round 6): one workgroup per CU forced by a dynamic-LDS floor on the decode launches.
#   base: as shipped; g: TI_GEMV_LDS_FLOOR=83968 (fused GEMV); ga: + TI_ATTN_LDS_PAD=65536 (attention)
# First the in-step stamp timeline of each arm (tools/stamp_probe.py: CU sharing, skews, gaps), then the
# default bench (configs[2]) interleaved twice per arm, then TinyLlama (configs[1]) once per arm.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6lds
mkdir -p $O
arm_env() {
  case $1 in
    base) echo "TI_NONE=0" ;;
    g) echo "TI_GEMV_LDS_FLOOR=83968" ;;
    ga) echo "TI_GEMV_LDS_FLOOR=83968 TI_ATTN_LDS_PAD=65536" ;;
  esac
}
show() {
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['calibration']['hbm_read_GBps'],{k:v['avg_us'] for k,v in d['kernels'].items()})" "$1" "$2"
}
for arm in base g ga; do
  env $(arm_env $arm) timeout -k 10 180 python3 tools/stamp_probe.py --json $O/stamp_$arm.json > $O/stamp_$arm.txt 2>&1 || { cat $O/stamp_$arm.txt; exit 1; }
  echo "== stamps $arm"; cat $O/stamp_$arm.txt
done
for r in 1 2; do
  for arm in base g ga; do
    env $(arm_env $arm) timeout -k 10 200 python3 bench.py --no-cpu-baseline --kernel-reps 20 > $O/b_${arm}_$r.json 2> $O/b_${arm}_$r.err || exit 1
    show $O/b_${arm}_$r.json "7b $arm $r"
  done
done
for arm in base g ga; do
  env $(arm_env $arm) timeout -k 10 200 python3 bench.py --model tinyllama-1.1b --no-cpu-baseline --kernel-reps 20 > $O/t_${arm}.json 2> $O/t_${arm}.err || exit 1
  show $O/t_${arm}.json "tl $arm"
done
