# PDS ring-depth A/B (TI_LIB builds in turboinfer_amd/lib/exp)
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in r4; do
  TI_LIB=turboinfer_amd/lib/exp/lib_$lib.so timeout -k 10 150 python3 tools/pds_phases.py > gpurun_out/pds_phases_$lib.txt 2>&1
  TI_LIB=turboinfer_amd/lib/exp/lib_$lib.so TI_PDS=1 timeout -k 10 200 python3 bench.py --steps 256 --no-cpu-baseline > gpurun_out/pds_ab_$lib.json 2> gpurun_out/pds_ab_$lib.err
done
