#!/bin/bash
# Round 6 GEMV fixed-cost changes: phase marks (lib_ph), bench, then the parity tests they touch.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6chk}
mkdir -p $O
PH=$GRAFT_REPO_ROOT/turboinfer_amd/lib_ph/libturboinfer_amd.so
TI_LIB=$PH timeout -k 10 180 python3 tools/stamp_probe.py --json $O/ph_7b.json > $O/ph_7b.txt 2>&1 || { cat $O/ph_7b.txt; exit 1; }
cat $O/ph_7b.txt
TI_LIB=$PH timeout -k 10 180 python3 tools/stamp_probe.py --model tinyllama-1.1b > $O/ph_tl.txt 2>&1 || { cat $O/ph_tl.txt; exit 1; }
cat $O/ph_tl.txt
for r in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench$r.json 2> $O/bench$r.err || { tail $O/bench$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench$r.json'));r=d['roofline'];print('bench',d['value'],d['calibration']['hbm_read_GBps'],r['frac'],r['span_frac'],r['isolated_frac'],r['avg_launch_us'],{k:(v['avg_us'],v['span_us']) for k,v in d['kernels'].items()})"
done
timeout -k 10 300 python3 bench.py --model tinyllama-1.1b --no-cpu-baseline > $O/bench_tl.json 2> $O/bench_tl.err || { tail $O/bench_tl.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_tl.json'));r=d['roofline'];print('bench tl',d['value'],r['frac'],{k:(v['avg_us'],v['span_us']) for k,v in d['kernels'].items()})"
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fold.py tests/test_gpu_kernels.py tests/test_gpu_g32.py "tests/test_gpu_deep.py::test_deep_llama2_7b_one_stream" "tests/test_gpu_deep.py::test_deep_tinyllama_one_stream" "tests/test_gpu_deep.py::test_deep_bench_replay" > $O/tests.txt 2>&1; rc=$?
tail -5 $O/tests.txt; cat $O/deep_parity.jsonl
exit $rc
