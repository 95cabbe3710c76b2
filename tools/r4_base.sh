#!/bin/bash
# Round-4 start: bench line (graph path) and the old persistent path, same box, plus a device-copy GB/s.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -c "
import torch,time
x=torch.empty(1<<30,dtype=torch.uint8,device='cuda'); y=torch.empty_like(x)
for _ in range(3): y.copy_(x)
torch.cuda.synchronize(); t=time.perf_counter()
for _ in range(20): y.copy_(x)
torch.cuda.synchronize(); dt=(time.perf_counter()-t)/20
print('copy GB/s (read+write)', 2*(1<<30)/dt/1e9)
" > gpurun_out/r4_copy.txt 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 16 --no-cpu-baseline > gpurun_out/r4_base_graph$i.json 2>gpurun_out/r4_base_graph$i.err || exit 1
TI_PDS=1 timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 16 --no-cpu-baseline > gpurun_out/r4_base_pds$i.json 2>gpurun_out/r4_base_pds$i.err || exit 1
done
