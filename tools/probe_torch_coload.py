"""Probe: can the product library (ROCm 7.2 HIP runtime) share a process with torch
(bundles its own ROCm 7.0 HIP runtime) when torch is only used for gloo coordination?
Prints which libamdhip64 copies are mapped and runs a tiny engine decode before and after."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
order = sys.argv[1] if len(sys.argv) > 1 else "lib_first"


def maps():
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l})


def run_engine(T):
    e = T.Engine(512, 256, 2, 4, 2, 64, 512, bits=4, max_seq=64, max_batch=1)
    e.synth(11, 0.1)
    out = e.generate([[1, 17, 42]], 4)
    e.close()
    return out[0].tolist()


if order == "torch_first":
    import torch
    import torch.distributed as dist
import turboinfer_amd as T

T.init(0)
print("tokens before torch:", run_engine(T))
if order == "lib_first":
    import torch
    import torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("gloo", rank=0, world_size=1)
t = torch.tensor([1.0])
dist.all_reduce(t, op=dist.ReduceOp.MAX)
dist.barrier()
print("gloo ok", t.item())
print("tokens after torch:", run_engine(T))
print("amdhip64 mapped:", maps())
dist.destroy_process_group()
