#!/bin/bash
# LDS bank conflicts of the decode kernels (configs[2] one stream, configs[3] 64 streams): one PMC pass each.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/ldspmc
mkdir -p $O
P="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES"
timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $O/c2 -o t -- python3 bench.py --steps 4 --warmup 2 --kernel-reps 4 --no-cpu-baseline > $O/c2.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $O/c3 -o t -- python3 bench.py --batch 64 --steps 4 --warmup 2 --kernel-reps 4 --no-cpu-baseline > $O/c3.log 2>&1 || exit 1
echo done
