"""Diagnostic: per-phase timeline of one persistent decode launch (TI_PDS_TS=1) at the bench's
7B configuration (32 layers, KV 2048, replay at position 2047).  Events per (workgroup, layer,
phase), s_memrealtime at 100 MHz: consumer 0 -- 0 phase start (gather begins), 1 input gathered
(after the consumer barrier), 2 consumed (after the barrier), 3 epilogue published (attention:
its split partial), 4 attention only: the head group's merged output published; loader -- 6 the
phase's first fill issue begins, 7 its last fill issued."""
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
t0 = t[:, 0, 0, 0].min()
names = ["QKV", "ATT", "O", "GU", "DN"]
print("err", e.pds_error())
print("launch span (us): %.1f  (%.2f per layer)" % ((t[:, NL - 1, 4, 3].max() - t0) / 100.0,
                                                   (t[:, NL - 1, 4, 3].max() - t0) / 100.0 / NL))
for p, nm in enumerate(names):
    sl = t[:, 1:, p, :]
    gat = (sl[..., 1] - sl[..., 0]) / 100.0
    con = (sl[..., 2] - sl[..., 1]) / 100.0
    epi = (sl[..., 3] - sl[..., 2]) / 100.0
    lead = (sl[..., 1] - sl[..., 6]) / 100.0    # consumers start - loader started the phase
    ltail = (sl[..., 2] - sl[..., 7]) / 100.0   # consumers done - loader issued the last fill
    extra = ""
    if nm == "ATT":
        extra = " merge %5.2f" % ((sl[..., 4] - sl[..., 3]) / 100.0).mean()
    print("%-4s gather %5.2f (max %5.2f) consume %5.2f (max %5.2f) epi %5.2f%s | loader lead %6.2f, done->consumed %5.2f" %
          (nm, gat.mean(), gat.max(axis=0).mean(), con.mean(), con.max(axis=0).mean(), epi.mean(), extra,
           lead.mean(), ltail.mean()))
pub = t[:, :, :, 3].copy()
pub[:, :, 1] = t[:, :, 1, 4]
last = pub.max(axis=0)  # [NL][5] last publish per phase
d = np.diff(last.reshape(-1)) / 100.0
print("critical-path increments (us, last publish of the phase after the previous one), mean over layers 1..:")
for p, nm in enumerate(names):
    idx = [l * 5 + p - 1 for l in range(1, NL)]
    print("  ->%-4s %.2f" % (nm, np.mean([d[i] for i in idx])))
print("per layer (us): %.2f" % (np.mean(np.diff(last[:, 4])) / 100.0))
e.close()
