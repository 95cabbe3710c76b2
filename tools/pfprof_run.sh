set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pfprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pfprof -o pf --output-format csv -- python3 tools/prefill_one.py 3 > gpurun_out/pfprof/log.txt 2>&1
