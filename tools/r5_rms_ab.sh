#!/bin/bash
# RECORD ONLY: the one-trip rms_norm was not kept (profiles/r5_rmsnorm_onetrip_ab.txt).
echo "the one-trip rms_norm was not kept (profiles/r5_rmsnorm_onetrip_ab.txt)"; exit 2
# rms_norm rows to fp16 in one round trip (row and weight held in registers across the reduction):
# the rms / batched / prefill / deep parity, then the 512-token prefill and the decode side configs,
# the previous commit's build (ablib/prev.so) against the new one, interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/rms
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_batched.py tests/test_gpu_prefill.py \
  tests/test_gpu_deep.py tests/test_gpu_engine.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for v in prev new; do
    case $v in prev) L=$PWD/ablib/prev.so;; new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; esac
    TI_LIB=$L timeout -k 10 200 python3 tools/prefill_bench.py 512 > $O/prefill_${v}_$r.txt 2>&1 || exit 1
    echo "$v run $r: $(grep 'rows 512' $O/prefill_${v}_$r.txt)"
  done
done
for v in prev new; do
  case $v in prev) L=$PWD/ablib/prev.so;; new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; esac
  TI_LIB=$L timeout -k 10 300 python3 bench.py --batch 64 --steps 16 --warmup 3 --no-cpu-baseline > $O/c3_$v.json 2> $O/e.txt || { tail $O/e.txt; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1]); print('$v c3', d['value'])"
done
