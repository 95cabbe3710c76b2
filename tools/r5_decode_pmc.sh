#!/bin/bash
# SQ / TA PMC passes over the one-stream decode (configs[2], short bench run): wait, VALU, MFMA and LDS shares
# of the fused GEMV and the attention.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/dpmc
mkdir -p $O
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAVES SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
i=0
for P in "$A" "$B"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o t -- python3 bench.py --steps 4 --warmup 2 --kernel-reps 4 --no-cpu-baseline > $O/p$i.log 2>&1 || exit 1
  echo "pass $i done"; tail -2 $O/p$i.log
done
python3 tools/r5_decode_pmc_sum.py $O > gpurun_out/dpmc_summary.txt
cat gpurun_out/dpmc_summary.txt
rm -rf $O
