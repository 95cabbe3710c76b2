#!/bin/bash
# Persistent decode with granule hand-offs: bit-identity to the per-layer launches, the fatal
# timeout path, then the bench with it on / off (interleaved) and the phase timeline.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pds.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pds_tests.log 2>&1
: > gpurun_out/pds_gran_ab.jsonl
for i in 1 2; do
  TI_PDS=1 timeout -k 10 200 python3 bench.py --steps 256 --no-cpu-baseline >> gpurun_out/pds_gran_ab.jsonl 2>> gpurun_out/pds_gran_ab.err
  timeout -k 10 200 python3 bench.py --steps 256 --no-cpu-baseline >> gpurun_out/pds_gran_ab.jsonl 2>> gpurun_out/pds_gran_ab.err
done
timeout -k 10 150 python3 tools/pds_phases.py > gpurun_out/pds_gran_phases.txt 2>&1
