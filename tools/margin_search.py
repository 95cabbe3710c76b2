"""Offline seed selection for the greedy parity tests (CPU, oracle only).

For a BASELINE config shape and weight seed, decodes every candidate stream (start token
(7 * seed + 13 * b) % V, KV seed 100 + b, synthetic cache of `fill` slots) for `steps`
steps in the oracle and prints the smallest top-2 margin / max|logit| over those steps.
The tests check streams whose margin exceeds 3x their logits tolerance, so that greedy
token equality follows from the logits bound.

  python3 tools/margin_search.py 7b 2025 64 2044 4
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from parity_probe import CFG  # noqa: E402
from pyoracle import Oracle, OracleModel  # noqa: E402


def main():
    name, seed, B, fill, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    cands = [int(x) for x in sys.argv[6].split(",")] if len(sys.argv) > 6 else range(B)
    cfg = CFG[name]
    V = cfg["vocab"]
    m = OracleModel(Oracle(), cfg, seed, 0.0)
    for b in cands:
        m.fill_kv(fill, 100 + b)
        t = (seed * 7 + 13 * b) % V
        mins = []
        for _ in range(steps):
            t, lg = m.step(t)
            s = np.sort(lg)
            mins.append(float(s[-1] - s[-2]) / float(np.max(np.abs(lg))))
        print(name, b, round(min(mins), 5), [round(x, 4) for x in mins], flush=True)


if __name__ == "__main__":
    main()
