#!/bin/bash
# Round 6: last split's shortening (TI_QA_EXTRA keys) of the fused QKV + attention launch with the new key attended
# in-launch: default (7B 32, TinyLlama 256) against other values, interleaved on one box
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/r6_ab.sh r6extra def=. x0=.,TI_QA_EXTRA=0 x64=.,TI_QA_EXTRA=64 x128=.,TI_QA_EXTRA=128 x384=.,TI_QA_EXTRA=384
