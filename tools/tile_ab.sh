# Prefill tile GEMM A/B at 256 rows (rows_bench), default build vs exp builds
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/rows_bench.py 256 > gpurun_out/tile_default.txt 2>&1
for lib in xb2; do
  TI_LIB=turboinfer_amd/lib/exp/lib_$lib.so timeout -k 10 200 python3 tools/rows_bench.py 256 > gpurun_out/tile_$lib.txt 2>&1
done
