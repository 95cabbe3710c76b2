# Persistent decode layers: bit-identity tests, phase timeline, then the bench with it on and off
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pds.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pds_tests.log 2>&1
timeout -k 10 150 python3 tools/pds_phases.py > gpurun_out/pds_phases.txt 2>&1
for i in 1; do
  TI_PDS=1 timeout -k 10 200 python3 bench.py --steps 256 --no-cpu-baseline > gpurun_out/pds_on_$i.json 2> gpurun_out/pds_on_$i.err
  TI_PDS=0 timeout -k 10 200 python3 bench.py --steps 256 --no-cpu-baseline > gpurun_out/pds_off_$i.json 2> gpurun_out/pds_off_$i.err
done
