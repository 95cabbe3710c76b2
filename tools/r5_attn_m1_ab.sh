#!/bin/bash
# RECORD ONLY: the one-stream ring stays 3 (profiles/r5_attn_m1_ring_ab.txt).
echo "the one-stream ring stays 3 (profiles/r5_attn_m1_ring_ab.txt)"; exit 2
# One-stream decode attention (configs[2]) with 2 / 3 (default) / 4 K/V ring slots per wave after the slot pinning:
# kernel / engine parity on the variants, then configs[2] bench lines interleaved x3.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/am1
mkdir -p $O
for v in m2 m4; do
  TI_LIB=$PWD/ablib/$v.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_kernels.py \
    -k attention > $O/tests_$v.txt 2>&1 || { tail -30 $O/tests_$v.txt; exit 1; }
  tail -1 $O/tests_$v.txt
done
for r in 1 2 3; do
  for v in new m2 m4; do
    case $v in new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; *) L=$PWD/ablib/$v.so;; esac
    TI_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/c2_${v}_$r.json 2> $O/e.txt || { tail $O/e.txt; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c2_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], 'attn GB/s', d['attention_roofline']['achieved'])"
  done
done
