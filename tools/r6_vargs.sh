#!/bin/bash
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/turboinfer_amd
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fold.py tests/test_gpu_kernels.py "tests/test_gpu_deep.py::test_deep_bench_replay" > gpurun_out/r6vargs_tests.txt 2>&1 || true
tail -2 gpurun_out/r6vargs_tests.txt
TI_LIB=$L/lib_vargs/libturboinfer_amd.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fold.py tests/test_gpu_kernels.py "tests/test_gpu_deep.py::test_deep_bench_replay" > gpurun_out/r6vargs_tests_v.txt 2>&1 || { tail -20 gpurun_out/r6vargs_tests_v.txt; exit 1; }
tail -2 gpurun_out/r6vargs_tests_v.txt
bash tools/r6_ab.sh r6vargs base=. vargs=$L/lib_vargs/libturboinfer_amd.so
