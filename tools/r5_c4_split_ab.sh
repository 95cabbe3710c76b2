#!/bin/bash
# configs[4] attention, two workgroups per CU: 2 splits per (stream, kv-head) = 512 workgroups on
# the 2-slot ring (tools/bin/rl2: TI_ATTN_RING_LONG=2, 124 VGPRs -> 2 x 8 waves per CU) vs the
# product (256 workgroups, 4-slot ring, 172 VGPRs, 1 per CU).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c4split
mkdir -p $O
run() {   # lib tag args...
  local lib=$1 tag=$2; shift 2
  L=""; [ $lib = prod ] || L=$GRAFT_REPO_ROOT/tools/bin/$lib/libturboinfer_amd.so
  TI_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --kernel-reps 20 --model llama3-8b --batch 32 --kv 8192 \
    --steps 32 --warmup 4 "$@" > $O/${tag}.json 2> $O/${tag}.err || exit 1
  python3 -c "import json;d=json.load(open('$O/${tag}.json'));print('$tag',d['value'],d['kernels']['attention']['avg_us'],d['kernels']['attention']['GBps'])"
}
for r in 1 2; do
  run prod prod_s1_$r
  run rl2 rl2_s2_$r --attn-splits 2
  run rl2 rl2_s1_$r --attn-splits 1
  run prod prod_s2_$r --attn-splits 2
done
