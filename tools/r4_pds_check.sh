#!/bin/bash
# Round 4: the loader-ring persistent decode (pds.hip) -- bit-identity tests first, then the whole
# GPU suite (chained / fused-QKV paths removed this round), bench A/B vs the graph, phase timeline.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pds.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_pds_tests.txt 2>&1
rc=$?
echo "pds tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 16 --no-cpu-baseline > gpurun_out/r4_graph1.json 2>gpurun_out/r4_graph1.err
echo "graph bench rc=$?"
TI_PDS=1 timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 16 --no-cpu-baseline > gpurun_out/r4_pds1.json 2>gpurun_out/r4_pds1.err
echo "pds bench rc=$?"
TI_PDS=1 TI_PDS_TS=1 timeout -k 10 200 python3 -u tools/pds_phases.py > gpurun_out/r4_pds_phases.txt 2>&1
echo "phases rc=$?"
# configs[4] attention A/B (tools/c4_attn_r4.sh variants): product vs rotated sweep vs 16 waves
: > gpurun_out/c4_attn_r4.txt
for v in base rot w16r2rot w16r2 base; do
  if [ $v = base ]; then L=""; else L=$GRAFT_REPO_ROOT/exp/$v/libturboinfer_amd.so; fi
  [ $v = base ] || [ -f "$L" ] || continue
  TI_LIB=$L timeout -k 10 200 python3 -u bench.py --model llama3-8b --batch 32 --kv 8192 --steps 16 --warmup 3 --no-cpu-baseline > gpurun_out/c4a_$v.json 2>> gpurun_out/c4_attn_r4.err || break
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/c4a_$v.json'));print(d['value'], d['ms_per_step'], d['kernels'].get('attention'))")" >> gpurun_out/c4_attn_r4.txt
done
echo "c4 ab done"
timeout -k 10 500 python3 -u -m pytest tests/ -q -m gpu --maxfail=10 --timeout 200 --timeout-method thread > gpurun_out/r4_suite.txt 2>&1
echo "suite rc=$?"
exit 0
