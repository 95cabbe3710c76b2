#!/bin/bash
# Round 6: the per-tile in-stream epilogue (TI_GEMV_EARLY) -- GEMV parity, the engine
# recipe probe, then the interleaved A/B against the build without it and the phase stamps.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6early
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_fold.py tests/test_gpu_engine.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
bash tools/r6_engine_probe.sh || exit 1
bash tools/r6_ab.sh r6early/ab cur=. ne=turboinfer_amd/lib_ne/libturboinfer_amd.so || exit 1
TI_LIB=turboinfer_amd/lib_ph/libturboinfer_amd.so timeout -k 10 180 python3 tools/stamp_probe.py > $O/ph_7b.txt 2>&1 || { cat $O/ph_7b.txt; exit 1; }
cat $O/ph_7b.txt
