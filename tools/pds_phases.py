"""Diagnostic: per-phase timeline of one persistent decode launch (TI_PDS_TS=1) at the bench's
7B configuration (32 layers, KV 2048, replay at position 2047)."""
import ctypes as C
import os
import sys

import numpy as np

os.environ["TI_PDS"] = "1"
os.environ["TI_PDS_TS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as ti

V, H, NL, NH, HD, I = 32000, 4096, 32, 32, 128, 11008
e = ti.Engine(V, H, NL, NH, NH, HD, I, bits=4, max_seq=2048, max_batch=1)
e.synth(0x7157, 0.1)
assert e.set_pds(True)
e.fill_kv(0, 2047, 0x5eed)
e.replay_prepare(1, 2048, 7)
e.replay_run(20)
e.sync()
n = 256 * NL * 5 * 8
buf = np.zeros(n, np.uint64)
ti.check(ti.lib().ti_engine_pds_timestamps(e.h, buf.ctypes.data_as(C.c_void_p), n))
t = buf.reshape(256, NL, 5, 8).astype(np.int64)
t0 = t[:, 0, 0, 2].min()
names = ["QKV", "ATT", "O", "GU", "DN"]
print("err", e.pds_error())
print("launch span (us): %.1f" % ((t[:, NL - 1, 4, 5].max() - t0) / 100.0))
# per phase, averaged over layers 1..NL-1 and workgroups: poll wait, staging, consume, epilogue
for p, nm in enumerate(names):
    sl = t[:, 1:, p, :]
    poll = (sl[..., 1] - sl[..., 0]) / 100.0
    stage = (sl[..., 2] - sl[..., 1]) / 100.0
    cons = (sl[..., 3] - sl[..., 2]) / 100.0
    b3 = (sl[..., 4] - sl[..., 3]) / 100.0
    epi = (sl[..., 5] - sl[..., 4]) / 100.0
    # critical path: last signal of this phase - last signal of the previous phase
    print("%-4s poll %5.2f stage %5.2f consume %5.2f (max %5.2f) wait-B3 %5.2f epi+signal %5.2f" %
          (nm, poll.mean(), stage.mean(), cons.mean(), cons.max(axis=0).mean(), b3.mean(), epi.mean()))
last = t[:, :, :, 5].max(axis=0)  # [NL][5] last signal per phase
seq = last.reshape(-1)
d = np.diff(seq) / 100.0
print("per-phase critical-path increments (us), mean over layers:")
for p, nm in enumerate(names):
    idx = [l * 5 + p - 1 for l in range(1, NL)]
    print("  ->%-4s %.2f" % (nm, np.mean([d[i] for i in idx])))
print("per layer (us): %.2f" % (np.mean(np.diff(last[:, 4])) / 100.0))
e.close()
