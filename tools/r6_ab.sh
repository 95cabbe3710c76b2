#!/bin/bash
# Interleaved A/B of library builds / knobs on one box: tools/ab_step.py per arm, 3 rounds.
#   bash tools/r6_ab.sh <out> <arm>=<lib path or ".">[,VAR=VAL...] ... [-- model ...]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
ARMS=(); MODELS=(llama2-7b tinyllama-1.1b)
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; MODELS=("$@"); break; fi
  ARMS+=("$1"); shift
done
for r in 1 2 3; do
  for m in "${MODELS[@]}"; do
    for a in "${ARMS[@]}"; do
      name=${a%%=*}; spec=${a#*=}
      lib=${spec%%,*}; envs=""; [ "$spec" != "$lib" ] && envs=${spec#*,}
      [ "$lib" = "." ] && lib=""
      env TI_LIB=$lib ${envs//,/ } timeout -k 10 120 python3 tools/ab_step.py --model $m --tag "$name r$r" >> $O/ab.txt 2>&1 || { tail -3 $O/ab.txt; exit 1; }
      tail -1 $O/ab.txt
    done
  done
done
python3 - $O/ab.txt <<'PY'
import re, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    m = re.match(r'(\S+) r\d (\S+) B=\d+ L=\d+: ([0-9.]+) tok/s', l)
    if m: d[(m.group(2), m.group(1))].append(float(m.group(3)))
for k, v in sorted(d.items()): print(*k, " ".join(f"{x:.1f}" for x in v), f"mean {sum(v) / len(v):.1f}")
PY
