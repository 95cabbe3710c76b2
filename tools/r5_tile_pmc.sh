#!/bin/bash
# PMC passes (one counter group per run) over the 7B QKV tile GEMM at 512 rows (tools/tile_one.py) and
# the prefill attention (tools/prefill_attn_time.py): what bounds the prefill kernels.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/tpmc
mkdir -p $O
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"
C="FETCH_SIZE TA_BUSY_avr"
D="TCC_HIT_sum TCC_MISS_sum TA_BUSY_max"
i=0
for P in "$A" "$B" "$C" "$D"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/tile$i -o t -- python3 tools/tile_one.py > $O/tile$i.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/attn$i -o t -- python3 tools/prefill_attn_time.py > $O/attn$i.log 2>&1 || exit 1
  echo "pass $i done"
done
