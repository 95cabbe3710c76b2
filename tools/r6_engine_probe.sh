#!/bin/bash
# the guide's engine recipe as a probe (tools/probe_engine.hip) beside the product step
# on the same box (tools/stamp_probe.py: in-step per-layer periods).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6eng
mkdir -p $O
/opt/rocm/bin/hipcc -std=c++20 -O3 --offload-arch=gfx950 -Iinclude -Iturboinfer_amd/csrc/kernels tools/probe_engine.hip -o /tmp/probe_engine || exit 1
timeout -k 10 90 /tmp/probe_engine 32 > $O/engine.txt 2>&1; rc=$?
cat $O/engine.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python3 tools/stamp_probe.py > $O/stamp.txt 2>&1 || { cat $O/stamp.txt; exit 1; }
cat $O/stamp.txt
