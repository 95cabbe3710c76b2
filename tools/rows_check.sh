set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in e128 e256; do TI_LIB=$PWD/turboinfer_amd/lib/libti_$v.so timeout -k 10 200 python3 -u tools/rows_bench.py 32 64 > gpurun_out/rows_$v.txt 2>&1; done
TI_GEMM_ROWS_RG=2 timeout -k 10 200 python3 -u tools/rows_bench.py 32 > gpurun_out/rows_rg2_32.txt 2>&1
