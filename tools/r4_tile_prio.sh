#!/bin/bash
# RECORD ONLY: TI_TILE_PRIO is no longer read by the library (profiles/r4_tile_prio_ab.txt); the script stops here.
echo "TI_TILE_PRIO is gone (profiles/r4_tile_prio_ab.txt)"; exit 2
# Tile GEMM: waves 4-7 at s_setprio 1 (abx/prio, -DTI_TILE_PRIO=1) vs the product build, one box,
# interleaved: per-kernel times (rocprofv3 over tools/tile_one.py, 7B shapes at 512 rows) and
# 512-token prefill; then the prefill tests under the variant.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/prio
mkdir -p $O
P=$GRAFT_REPO_ROOT/abx/prio/libturboinfer_amd.so
for rep in 1 2; do
  for v in base prio; do
    if [ $v = prio ]; then export TI_LIB=$P; else unset TI_LIB; fi
    for shape in "512 12288 4096" "512 22016 4096" "512 4096 11008" "512 4096 4096"; do
      tag=${v}${rep}_$(echo $shape | tr ' ' _)
      timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag -o t -- python3 tools/tile_one.py $shape 20 > $O/$tag.log 2>&1
    done
    echo "$v $rep" >> $O/prefill.txt
    timeout -k 10 200 python3 tools/prefill_bench.py 512 >> $O/prefill.txt 2>&1
  done
done
TI_LIB=$P timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill.py "tests/test_gpu_deep.py::test_deep_prefill_then_decode" -x -q --timeout 150 --timeout-method thread > $O/tests.txt 2>&1
