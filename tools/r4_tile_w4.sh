#!/bin/bash
# Prefill tile GEMM on 4-wave workgroups (128-row waves, TI_TILE_W4=2|3) vs the 8-wave plans:
# parity (prefill + deep prefill tests under each knob), per-kernel times (rocprofv3 stats over
# tools/tile_one.py for the 7B shapes at 512 rows), and 512-token prefill end to end.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/w4
mkdir -p $O
for w in 2 3; do
  TI_TILE_W4=$w timeout -k 10 300 python3 -u -m pytest tests/test_gpu_prefill.py tests/test_gpu_prefill_attn.py \
    "tests/test_gpu_deep.py::test_deep_prefill_then_decode" -x -q --timeout 150 --timeout-method thread > $O/tests_w$w.txt 2>&1
done
for w in 0 2 3; do
  for shape in "512 12288 4096" "512 22016 4096" "512 4096 11008" "512 4096 4096" "1024 12288 4096"; do
    tag=w${w}_$(echo $shape | tr ' ' _)
    TI_TILE_W4=$w timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag -o t -- python3 tools/tile_one.py $shape 20 > $O/$tag.log 2>&1
  done
done
for w in 0 2 3 0 2 3; do
  echo "W4=$w" >> $O/prefill.txt
  TI_TILE_W4=$w timeout -k 10 200 python3 tools/prefill_bench.py 512 >> $O/prefill.txt 2>&1
done
