#!/bin/bash
# RECORD ONLY: TI_ATTN_BLOCK lost this A/B (profiles/r5_attn_block_ab.txt) and its code was removed afterwards, so on
# this tree both arms would be the same build; the script stops here.
echo "TI_ATTN_BLOCK was removed after this A/B (profiles/r5_attn_block_ab.txt)"; exit 2
# Blocked online softmax in the decode attention (TI_ATTN_BLOCK=1, product) vs per key
# (tools/bin/ab0, TI_ATTN_BLOCK=0): parity suites of the attention consumers first, then the four
# bench configurations interleaved (A B A B).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/attn_ab
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py tests/test_gpu_deep.py \
  tests/test_gpu_fold.py tests/test_gpu_batched.py -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
echo "tests rc=$?" >> $O/tests.txt; tail -3 $O/tests.txt
run() {   # arm tag args...
  local arm=$1 tag=$2; shift 2
  L=""; [ $arm = b1 ] || L=$GRAFT_REPO_ROOT/tools/bin/$arm/libturboinfer_amd.so
  TI_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --kernel-reps 20 "$@" > $O/${tag}_${arm}.json 2> $O/${tag}_${arm}.err || exit 1
  python3 -c "import json;d=json.load(open('$O/${tag}_${arm}.json'));print('$tag','$arm',d['value'],d['kernels']['attention']['avg_us'],d['kernels']['attention']['GBps'])"
}
for r in 1 2; do
  for arm in b1 ab0; do
    run $arm c4_$r --model llama3-8b --batch 32 --kv 8192 --steps 32 --warmup 4
    run $arm c3_$r --batch 64 --steps 32 --warmup 4
    run $arm c2_$r
  done
done
for arm in b1 ab0; do run $arm c1 --model tinyllama-1.1b; done
