#!/bin/bash
# Kernel trace of the 512-token prefill (tools/prefill_one.py: one 512-row chunk, 3 timed reps).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pfprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pfprof -o pf -- python3 tools/prefill_one.py 3 > gpurun_out/pfprof/run.log 2>&1
