#!/bin/bash
# Batched configs (configs[3]: 64 x 7B, configs[4]: 32 x Llama-3-8B @ 8192) product vs a variant
# library tools/bin/<arm>/ (built with make BUILD=build_<arm> LIB=tools/bin/<arm>/libturboinfer_amd.so
# EXTRA=-D...), interleaved A B A B; then one FETCH_SIZE pass of configs[3] on the variant.
#   bash tools/r5_batched_ab.sh <arm>
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
ARM=$1
O=gpurun_out/bab_$ARM
mkdir -p $O
run() {   # lib tag args...
  local lib=$1 tag=$2; shift 2
  L=""; [ $lib = prod ] || L=$GRAFT_REPO_ROOT/tools/bin/$lib/libturboinfer_amd.so
  TI_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --kernel-reps 20 --steps 32 --warmup 4 "$@" \
    > $O/${tag}_$lib.json 2> $O/${tag}_$lib.err || exit 1
  python3 -c "import json;d=json.load(open('$O/${tag}_$lib.json'));print('$tag','$lib',d['value'],{k:v['avg_us'] for k,v in d['kernels'].items()})"
}
for r in 1 2; do
  for lib in prod $ARM; do
    run $lib c3_$r --batch 64
    run $lib c4_$r --model llama3-8b --batch 32 --kv 8192
  done
done
TI_LIB=$GRAFT_REPO_ROOT/tools/bin/$ARM/libturboinfer_amd.so DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -s KILL 200 \
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_c3 -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --kernel-reps 4 --no-cpu-baseline --batch 64 > $O/pmc_c3.log 2>&1
echo "pmc rc=$?"
