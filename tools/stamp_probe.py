#!/usr/bin/env python3
"""In-step launch timeline of the replay step (ti_engine_stamp_steps), summarised per launch class.

    python tools/stamp_probe.py [--model llama2-7b] [--batch 1] [--kv 2048] [--steps 20] [--json out.json]

Per class (tag): launches per step, mean span / period / entry skew / wave-end skew / tail / gap (us)
and the mean count of workgroups that shared a CU with another workgroup of the same launch; the
sum of periods against the wall-clock step time of the same engine (graph replays back to back)."""
from __future__ import annotations

import argparse
import json
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
    ap.add_argument("--kv", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--seed", type=int, default=0x7157)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    import turboinfer_amd as T
    T.init(0)
    V, H, layers, nh, nkv, hd, I, bits, theta = MODELS[args.model]
    B, L = args.batch, args.kv
    e = T.Engine(V, H, layers, nh, nkv, hd, I, bits=bits, max_seq=L, max_batch=B, rope_theta=theta)
    e.synth(args.seed, 0.0)
    for s in range(B):
        e.fill_kv(s, L - 1, args.seed + s)
    e.replay_prepare(B, L, args.seed % V)
    e.replay_run(16)
    e.sync()
    t0 = time.perf_counter()
    e.replay_run(128)
    e.sync()
    step_us = (time.perf_counter() - t0) / 128 * 1e6
    launches = e.stamp_steps(args.steps)
    e.close()
    classes = {}
    for d in launches:
        c = classes.setdefault(d["tag"], {"kind": d["kind"], "n": 0, "workgroups": d["workgroups"]})
        c["n"] += 1
        for k in T.Engine.STAMP_FIELDS:
            c[k] = c.get(k, 0.0) + d[k]
    print(f"{args.model} B={B} L={L}: step {step_us:.1f} us wall (back to back), {len(launches)} launches, "
          f"sum of periods {sum(d['period_us'] for d in launches):.1f} us (one stamped step alone)")
    print(f"{'class':10s} {'kind':10s} {'n':>4s} {'wgs':>5s} " + " ".join(f"{k[:-3] if k.endswith('_us') else k:>12s}"
                                                                     for k in T.Engine.STAMP_FIELDS))
    for tag, c in classes.items():
        print(f"{tag:10s} {c['kind']:10s} {c['n']:4d} {c['workgroups']:5d} " +
              " ".join(f"{c[k] / c['n']:12.3f}" for k in T.Engine.STAMP_FIELDS))
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"model": args.model, "batch": B, "kv": L, "step_us_wall": step_us, "launches": launches}, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
