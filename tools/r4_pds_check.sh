#!/bin/bash
# Round 4: the loader-ring persistent decode (pds.hip) -- bit-identity tests, bench A/B vs the graph,
# phase timeline; then the round's new parity tests (prefill at full depth, generate() contract).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 16 --no-cpu-baseline > gpurun_out/r4_graph1.json 2>gpurun_out/r4_graph1.err || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pds.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_pds_tests.txt 2>&1
rc=$?
echo "pds tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TI_PDS=1 timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 16 --no-cpu-baseline > gpurun_out/r4_pds1.json 2>gpurun_out/r4_pds1.err
echo "pds bench rc=$?"
TI_PDS=1 TI_PDS_TS=1 timeout -k 10 200 python3 -u tools/pds_phases.py > gpurun_out/r4_pds_phases.txt 2>&1
echo "phases rc=$?"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_deep.py -k prefill tests/test_cpp_api.py -k "prefill or contract" -v --timeout 200 --timeout-method thread > gpurun_out/r4_new_tests.txt 2>&1
echo "new tests rc=$?"
exit 0
