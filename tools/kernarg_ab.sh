set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/kernarg_ab.txt
for v in unset 1 0 unset 1 0; do
  if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
  timeout -k 10 300 python3 -u bench.py --steps 128 --warmup 8 --no-cpu-baseline > gpurun_out/ka.json 2>> gpurun_out/ka.err
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/ka.json'));print(d['value'], d['ms_per_step'])")" >> gpurun_out/kernarg_ab.txt
done
