#!/bin/bash
# SQ counter passes over tools/prefill_attn_time.py (the prefill attention alone): wait / VALU / MFMA shares.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pfpmc
mkdir -p $O
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
i=0
for P in "$A" "$B"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o t -- python3 tools/prefill_attn_time.py > $O/p$i.log 2>&1 || exit 1
  echo "pass $i done"
done
python3 tools/r5_decode_pmc_sum.py $O > gpurun_out/pfpmc_summary.txt
cat gpurun_out/pfpmc_summary.txt
rm -rf $O
