#!/bin/bash
# Round-4 end (b): batched fold A/B, then the profile of the product bench line.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/r4_fold_ab.sh || exit 1
echo "fold ab done"
bash tools/r4_profile.sh r4 || exit 1
echo "profile done"
