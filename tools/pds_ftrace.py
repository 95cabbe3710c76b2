"""Diagnostic: per-fill ring events of the persistent decode launch (exp build with
-DTI_PDS_FTRACE=1, run with TI_LIB pointing at it) for workgroups 0..3 at the bench's 7B
configuration.  Events per fill (s_memrealtime, 100 MHz): 0 loader issue begins, 1 published
(FULL > fill), 2 consumer 0's wait ends, 3 consumer 0 releases it, 4/5 the loader's wait for a
FREE slot before issuing it (start / end), 6 its last piece issued.  DETAIL=0 skips the per-fill
listing."""
import ctypes as C
import os
import sys

import numpy as np

os.environ["TI_PDS"] = "1"
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
L = ti.lib()
L.ti_pds_ftrace.argtypes = [C.c_void_p, C.c_size_t]
buf = np.zeros(4 * 2048 * 8, np.uint64)
ti.check(L.ti_pds_ftrace(buf.ctypes.data_as(C.c_void_p), buf.size))
e.close()
tr = buf.reshape(4, 2048, 8).astype(np.int64)
KT_H, KT_Q, KT_I = H // 128, H // 128, I // 128
names = ["QKV", "ATT", "O", "GU", "DN"]
for b in range(4):
    gun = (b + 1) * (2 * I // 16) // 256 - b * (2 * I // 16) // 256
    items = [3 * KT_H, None, KT_Q, gun * KT_H, KT_I]
    nf = [-(-it // 16) if it else 8 for it in items]   # ATT: 2 * 64 pieces = 8 fills
    per_layer = sum(nf)
    t = tr[b]
    n = per_layer * NL
    t0 = t[0, 0]
    print(f"wg {b}: fills per layer {nf} = {per_layer}; launch {(t[n - 1, 3] - t0) / 100:.1f} us")
    for ph in range(5):
        idx = []
        for l in range(2, NL):
            base = l * per_layer + sum(nf[:ph])
            idx += list(range(base, base + nf[ph]))
        idx = np.array(idx)
        ev = t[idx]
        pub_lat = (ev[:, 1] - ev[:, 0]) / 100
        cons_lag = (ev[:, 2] - ev[:, 1]) / 100
        hold = (ev[:, 3] - ev[:, 2]) / 100
        blocked = ev[:, 4] > 0
        blk = ((ev[:, 5] - ev[:, 4]) / 100)[blocked]
        # cadence: issue of fill k+1 - issue of fill k, within the phase
        cad = np.diff(t[idx, 0]) / 100
        idur = (ev[:, 6] - ev[:, 0]) / 100
        math = ((ev[:, 7] - ev[:, 3]) / 100)[ev[:, 7] > 0] if ph != 1 else np.zeros(1)
        gapv = np.diff(ev[:, 2]) / 100   # consumer 0: acquire to next acquire within the phase
        print(f"  {names[ph]:4s} issue {idur.mean():5.2f}  issue->pub {pub_lat.mean():5.2f}  pub->acq {cons_lag.mean():6.2f}  acq->rel {hold.mean():5.2f}"
              f"  issue cadence {np.median(cad):5.2f}  blocked {blocked.mean()*100:4.0f}% ({blk.mean() if blk.size else 0:5.2f} us)"
              f"  acq-issue {((ev[:, 2] - ev[:, 0]) / 100).mean():6.2f}  rel->math {math.mean():5.2f}"
              f"  acq cadence {np.median(gapv) if gapv.size else 0:5.2f}")
    # one layer in detail (layer 5): fill, issue, pub, acq, rel relative to the layer's first issue
    if os.environ.get("DETAIL", "1") == "0":
        break
    l = 5
    base = l * per_layer
    tl0 = t[base, 0]
    print("  layer 5 detail (us from its first issue): fill phase issue pub acq rel [block]")
    k = 0
    for ph in range(5):
        for j in range(nf[ph]):
            ev = t[base + k]
            blk = f" blk {(ev[4] - tl0) / 100:6.2f}-{(ev[5] - tl0) / 100:6.2f}" if ev[4] else ""
            print(f"    {k:3d} {names[ph]:4s} {(ev[0] - tl0) / 100:7.2f} {(ev[1] - tl0) / 100:7.2f} {(ev[2] - tl0) / 100:7.2f} {(ev[3] - tl0) / 100:7.2f}{blk}")
            k += 1
    if b >= 1:
        break
