# TinyLlama INT8 one-stream attention: split count x head-parallel ring depth
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in nohp nohp_r4; do
  for sp in 0 8 16; do
    TI_LIB=turboinfer_amd/lib/exp/lib_$lib.so timeout -k 10 200 python bench.py --model tinyllama-1.1b --steps 256 --no-cpu-baseline --attn-splits $sp > gpurun_out/tl_${lib}_sp$sp.json 2> gpurun_out/tl_${lib}_sp$sp.err
  done
done
