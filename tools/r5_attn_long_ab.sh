#!/bin/bash
# RECORD ONLY: the long-range ring stays 4 (profiles/r5_attn_long_ring_ab.txt).
echo "the long-range ring stays 4 (profiles/r5_attn_long_ring_ab.txt)"; exit 2
# Long-range decode attention (configs[4]: one workgroup per (stream, kv-head), 8192 keys) with a K/V ring of
# 4 (default) / 6 / 8 slots per wave now that the ring's slots are pinned: Llama-3 parity on each, then
# configs[4] bench lines interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/along
mkdir -p $O
for v in al6 al8; do
  TI_LIB=$PWD/ablib/$v.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_engine.py \
    -k "llama3 or 8192 or gqa" > $O/tests_$v.txt 2>&1 || { tail -30 $O/tests_$v.txt; exit 1; }
  tail -1 $O/tests_$v.txt
done
for r in 1 2; do
  for v in new al6 al8; do
    case $v in new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; *) L=$PWD/ablib/$v.so;; esac
    TI_LIB=$L timeout -k 10 300 python3 bench.py --model llama3-8b --batch 32 --kv 8192 --steps 16 --warmup 3 --no-cpu-baseline \
      > $O/c4_${v}_$r.json 2> $O/e.txt || { tail $O/e.txt; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c4_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], 'attn GB/s', d['attention_roofline']['achieved'])"
  done
done
