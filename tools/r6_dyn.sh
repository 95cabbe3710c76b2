#!/bin/bash
# DYN (dynamic item claiming) parity + A/B against the static deal (TI_GEMV_DYN=0) and deeper rings.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6dyn
mkdir -p $O
L=$GRAFT_REPO_ROOT/turboinfer_amd
TI_PARITY_LOG=$O/deep_parity.jsonl timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fold.py tests/test_gpu_kernels.py tests/test_gpu_g32.py "tests/test_gpu_deep.py::test_deep_llama2_7b_one_stream" "tests/test_gpu_deep.py::test_deep_tinyllama_one_stream" "tests/test_gpu_deep.py::test_deep_bench_replay" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt; cat $O/deep_parity.jsonl
TI_LIB=$L/lib_ph/libturboinfer_amd.so timeout -k 10 180 python3 tools/stamp_probe.py > $O/ph_7b.txt 2>&1 || { cat $O/ph_7b.txt; exit 1; }
cat $O/ph_7b.txt
bash tools/r6_ab.sh r6dyn static=.,TI_GEMV_DYN=0 dyn=. ring24=$L/lib_ring24/libturboinfer_amd.so ring32=$L/lib_ring32/libturboinfer_amd.so
