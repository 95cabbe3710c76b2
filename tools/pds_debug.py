"""Diagnostic: persistent decode layers vs per-layer launches, max |diff| of logits per step;
pairs (on, off), (on, on), (off, off) to separate races from arithmetic differences."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as ti

cfg = (512, 256, 2, 2, 2, 128, 512)
v, h, l, nh, nkv, hd, inter = cfg
for pair in ((True, False), (True, True), (False, False)):
    eng = []
    for on in pair:
        e = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=4, max_seq=256, max_batch=1, attn_splits=8)
        e.synth(0x7157, 0.1)
        e.set_prefill(0)
        e.set_fold(True)
        e.set_pds(on)
        eng.append(e)
    toks = [3, 17, 99, 5]
    bad = []
    for pos in range(60):
        a = eng[0].step([toks[pos]], [pos])[0]
        b = eng[1].step([toks[pos]], [pos])[0]
        if not np.array_equal(a.view(np.uint32), b.view(np.uint32)):
            bad.append((pos, float(np.abs(a - b).max())))
        if pos + 1 >= len(toks):
            toks.append(int(np.argmax(b)))
    print(pair, "mismatching steps:", bad, "err", [e.pds_error() for e in eng], flush=True)
    for e in eng:
        e.close()
