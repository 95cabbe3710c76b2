set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/rows_bench.py 64 128 256 > gpurun_out/rows_tile.txt 2>&1
timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/prefill.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pf -o pf -- python3 tools/prefill_bench.py > gpurun_out/prefill_prof.log 2>&1
