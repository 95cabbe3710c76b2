"""Measure the decode engine's logit error against the oracle at the BASELINE configs' shapes
(2 layers each), per stream and step, to size the test tolerances.

  python3 tools/parity_probe.py [7b1|7b64|l3|tl|all]

Prints one JSON line per (config, stream, step): err / max|ref|, the oracle's top-2 margin /
max|ref| and whether the greedy tokens agree."""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import turboinfer_amd as T  # noqa: E402
from pyoracle import Oracle, OracleModel  # noqa: E402

CFG = {
    "7b": dict(vocab=32000, hidden=4096, layers=2, heads=32, kv_heads=32, head_dim=128, inter=11008,
               rope_theta=10000.0, eps=1e-5, bits=4, group=128, max_seq=2048),
    "l3": dict(vocab=128256, hidden=4096, layers=2, heads=32, kv_heads=8, head_dim=128, inter=14336,
               rope_theta=500000.0, eps=1e-5, bits=4, group=128, max_seq=8192),
    "tl": dict(vocab=32000, hidden=2048, layers=2, heads=32, kv_heads=4, head_dim=64, inter=5632,
               rope_theta=10000.0, eps=1e-5, bits=8, group=128, max_seq=2048),
}


def probe(name, cfg, seed, B, checked, n_steps):
    fill = cfg["max_seq"] - n_steps
    V = cfg["vocab"]
    toks0 = [(seed * 7 + 13 * b) % V for b in range(B)]
    e = T.Engine(cfg["vocab"], cfg["hidden"], cfg["layers"], cfg["heads"], cfg["kv_heads"], cfg["head_dim"],
                 cfg["inter"], bits=cfg["bits"], max_seq=cfg["max_seq"], max_batch=B, rope_theta=cfg["rope_theta"],
                 eps=cfg["eps"])
    e.synth(seed, 0.0)
    for b in range(B):
        e.fill_kv(b, fill, 100 + b)
    got = []
    toks = list(toks0)
    for s in range(n_steps):
        lg = e.step(toks, [fill + s] * B)
        got.append(lg[checked].copy())
        toks = [int(t) for t in np.argmax(lg, axis=1)]
    for b in range(B):
        e.fill_kv(b, fill, 100 + b)
    gen = e.generate([[t] for t in toks0], n_steps, start_pos=[fill] * B)
    e.close()
    m = OracleModel(Oracle(), cfg, seed, 0.0)
    for i, b in enumerate(checked):
        m.fill_kv(fill, 100 + b)
        t = toks0[b]
        for s in range(n_steps):
            t, lg = m.step(t)
            mx = float(np.max(np.abs(lg)))
            srt = np.sort(lg)
            err = float(np.max(np.abs(got[s][i].astype(np.float64) - lg)))
            l2 = float(np.linalg.norm(got[s][i] - lg) / np.linalg.norm(lg))
            print(json.dumps(dict(cfg=name, B=B, stream=b, step=s, err_rel_max=err / mx, l2_rel=l2,
                                  margin_rel_max=float(srt[-1] - srt[-2]) / mx, maxabs=mx,
                                  tok_ref=int(t), tok_gen=int(gen[b, s]), step_argmax=int(np.argmax(got[s][i])))),
                  flush=True)
    m.close()


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    T.init(0)
    if which in ("7b1", "all"):
        probe("7b", CFG["7b"], 2025, 1, [0], 4)
    if which in ("tl", "all"):
        probe("tl", CFG["tl"], 1101, 1, [0], 4)
    if which in ("7b64", "all"):
        probe("7b", CFG["7b"], 2025, 64, [0, 21, 42, 63], 4)
    if which in ("l3", "all"):
        probe("l3", CFG["l3"], 808, 32, [0, 13, 31], 3)
