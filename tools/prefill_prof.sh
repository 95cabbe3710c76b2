# Prefill: timing and a kernel-trace profile (7B INT4, 512-token prompt)
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/prefill.txt 2>&1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pf -o pf -- python3 tools/prefill_bench.py > gpurun_out/prefill_prof.log 2>&1
