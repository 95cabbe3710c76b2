#!/bin/bash
# HIP runtime environment knobs against the graph's kernel-to-kernel gap (7B decode step)
cd $GRAFT_REPO_ROOT
bash tools/r6_ab.sh r6env base=. sss0=.,ROC_SYSTEM_SCOPE_SIGNAL=0 dd0=.,AMD_DIRECT_DISPATCH=0 dd1=.,AMD_DIRECT_DISPATCH=1 fgs0=.,ROC_USE_FGS_KERNARG=0 devk=.,HIP_FORCE_DEV_KERNARG=1 -- llama2-7b
