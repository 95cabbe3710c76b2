#!/bin/bash
# Affine group-32 (GGUF Q4_1) kernels, engine and C++ API on the GPU, plus the group-32 / kernel suites around them.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_g32.py -x -v --timeout 120 --timeout-method thread > gpurun_out/q41_g32.log 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_cpp_api.py -x -v -m gpu -k "gguf or q_blocks" --timeout 120 --timeout-method thread > gpurun_out/q41_cpp.log 2>&1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q41_kernels.log 2>&1
