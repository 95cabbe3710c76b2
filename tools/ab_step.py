#!/usr/bin/env python3
"""Decode step throughput of the replay step (the bench's timed region) with whatever library TI_LIB
names -- old builds included (only the round-1 engine API is used): A/B runs interleave builds.

    TI_LIB=... python tools/ab_step.py [--model llama2-7b] [--batch 1] [--steps 256]"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import MODELS  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b", choices=sorted(MODELS))
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--kv", type=int, default=0)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import turboinfer_amd as T
    T.init(0)
    V, H, layers, nh, nkv, hd, I, bits, theta = MODELS[args.model]
    B = args.batch
    L = args.kv or (8192 if args.model == "llama3-8b" else 2048)
    e = T.Engine(V, H, layers, nh, nkv, hd, I, bits=bits, max_seq=L, max_batch=B, rope_theta=theta)
    e.synth(0x7157, 0.0)
    for s in range(B):
        e.fill_kv(s, L - 1, 0x7157 + s)
    e.replay_prepare(B, L, 0x7157 % V)
    e.replay_run(16)
    e.sync()
    t0 = time.perf_counter()
    e.replay_run(args.steps)
    e.sync()
    dt = time.perf_counter() - t0
    e.close()
    print(f"{args.tag} {args.model} B={B} L={L}: {B * args.steps / dt:.1f} tok/s, {dt / args.steps * 1e6:.1f} us/step")
    return 0


if __name__ == "__main__":
    sys.exit(main())
