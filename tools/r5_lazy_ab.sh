#!/bin/bash
# RECORD ONLY: TI_ATTN_LAZY lost this A/B (profiles/r5_attn_lazy_ab.txt) and was reverted; the script stops here.
echo "TI_ATTN_LAZY was reverted (profiles/r5_attn_lazy_ab.txt)"; exit 2
# Lazy running-max rescale in the decode attention (TI_ATTN_LAZY=1 build in tools/bin/lazy/): attention /
# engine / deep parity with the variant library, then the bench lines of configs[2], [1], [3], [4]
# per arm (attention kernel times from the lines' kernels field).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/lazy
mkdir -p $O
S=$GRAFT_REPO_ROOT/tools/bin/lazy/libturboinfer_amd.so
TI_LIB=$S timeout -k 10 600 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_kernels.py -k attention tests/test_gpu_engine.py tests/test_gpu_deep.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do
  for arm in base lazy; do
    L=""; [ $arm = lazy ] && L=$S
    TI_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/c2_${arm}_$r.json 2>/dev/null || exit 1
    TI_LIB=$L timeout -k 10 200 python3 bench.py --model tinyllama-1.1b --no-cpu-baseline > $O/c1_${arm}_$r.json 2>/dev/null || exit 1
    TI_LIB=$L timeout -k 10 300 python3 bench.py --batch 64 --steps 16 --warmup 3 --no-cpu-baseline > $O/c3_${arm}_$r.json 2>/dev/null || exit 1
    TI_LIB=$L timeout -k 10 300 python3 bench.py --model llama3-8b --batch 32 --kv 8192 --steps 16 --warmup 3 --no-cpu-baseline > $O/c4_${arm}_$r.json 2>/dev/null || exit 1
    for c in c2 c1 c3 c4; do
      python3 -c "import json;d=json.load(open('$O/${c}_${arm}_$r.json'));print('$c $arm $r', d['value'], d['kernels']['attention']['avg_us'])"
    done
  done
done
