#!/bin/bash
# PMC passes over the tile GEMM (7B QKV, 512 rows): wave-cycle split and instruction mix.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tile_pmc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/tile_pmc/trace -o trace -- python3 tools/tile_one.py > gpurun_out/tile_pmc/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES -d gpurun_out/tile_pmc/p1 -o p1 -- python3 tools/tile_one.py > gpurun_out/tile_pmc/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/tile_pmc/p2 -o p2 -- python3 tools/tile_one.py > gpurun_out/tile_pmc/p2.log 2>&1
