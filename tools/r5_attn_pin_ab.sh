#!/bin/bash
# Decode attention with its K/V ring slots pinned in order (ring_pin) and q loaded before the ring:
# attention / engine / deep parity on the new build, then bench lines (configs[2], [4], [1], [3]) with the
# per-class attention time for the round-5 build (ablib/old.so) and the new one, interleaved.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/apin
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_batched.py tests/test_gpu_engine.py tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for v in old new; do
    case $v in old) L=$PWD/ablib/old.so;; new) L=$PWD/turboinfer_amd/lib/libturboinfer_amd.so;; esac
    : > $O/b_${v}_$r.jsonl
    TI_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline >> $O/b_${v}_$r.jsonl 2> $O/e.txt || { tail $O/e.txt; exit 1; }
    TI_LIB=$L timeout -k 10 300 python3 bench.py --model llama3-8b --batch 32 --kv 8192 --steps 16 --warmup 3 --no-cpu-baseline >> $O/b_${v}_$r.jsonl 2> $O/e.txt || { tail $O/e.txt; exit 1; }
    TI_LIB=$L timeout -k 10 300 python3 bench.py --model tinyllama-1.1b --no-cpu-baseline >> $O/b_${v}_$r.jsonl 2> $O/e.txt || { tail $O/e.txt; exit 1; }
    TI_LIB=$L timeout -k 10 300 python3 bench.py --batch 64 --steps 16 --warmup 3 --no-cpu-baseline >> $O/b_${v}_$r.jsonl 2> $O/e.txt || { tail $O/e.txt; exit 1; }
    python3 - $O/b_${v}_$r.jsonl $v $r <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    a = d.get("per_class", d.get("kernels", {}))
    att = d.get("attention_roofline", {})
    print(sys.argv[2], sys.argv[3], d["config"].get("workload", "")[:40], d["value"], "attn GB/s", att.get("achieved"))
PY
  done
done
