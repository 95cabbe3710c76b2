"""Long greedy runs at full depth ("drift over a longer greedy run at full depth
is unmeasured"): the deep fixtures of gen_deep.py hold three steps per stream; these hold
N_LONG = 64 greedy steps of one stream per config, from the full-depth oracle
(oracle/ti_oracle_deep.c, bit-identical to the pinned or_decode_step: tests/test_oracle_deep.py).

Per config: the synthetic model of gen_deep.py (same engine seed, unit norms), the stream's KV cache
filled with synthetic fp16 rows up to max_seq - N_LONG, then N_LONG greedy decode steps from tok0,
the last at max_seq - 1.  Every step after the first attends over the cache rows the run itself
wrote, so an error in K/V written at step i reaches every later step.

Stored per step: the greedy token, the top-2 margin, max|logit| and the TOPK largest logits (index,
value); the full fp32 logits at the steps in FULL_AT.  (All 64 full logit vectors would be 8 MB per
config; the top-k set holds every entry a greedy or top-k sampler reads.)

    python tests/golden/gen_deep_long.py                # both configs (~3 min, 8 threads)
    python tests/golden/gen_deep_long.py tinyllama_1b   # one config
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)
from gen_deep import CONFIGS  # noqa: E402
from pyoracle import Oracle, OracleDeepModel  # noqa: E402

N_LONG = 64
TOPK = 16
FULL_AT = (0, 1, 15, 31, 47, 63)

# name -> (tok0, kv_seed) of the long stream
STREAMS = {"llama2_7b": (4321, 100), "tinyllama_1b": (2718, 101)}


def make(name: str, oracle: Oracle) -> None:
    what, cfg, seed, _ = CONFIGS[name]
    tok0, kv_seed = STREAMS[name]
    t0 = time.time()
    m = OracleDeepModel(oracle, cfg, seed, 0.0)
    fill = cfg["max_seq"] - N_LONG
    m.fill_kv(fill, kv_seed)
    toks, top_i, top_v, marg, mx, full = [], [], [], [], [], []
    t = tok0
    for step in range(N_LONG):
        t, lg = m.step(t)
        toks.append(t)
        idx = np.argsort(lg, kind="stable")[::-1][:TOPK]
        top_i.append(idx.astype(np.int32))
        top_v.append(lg[idx].astype(np.float32))
        marg.append(float(lg[idx[0]] - lg[idx[1]]))
        mx.append(float(np.abs(lg).max()))
        if step in FULL_AT:
            full.append(lg.astype(np.float32))
    m.close()
    marg, mx = np.array(marg, np.float32), np.array(mx, np.float32)
    out = dict(cfg=np.array(json.dumps(cfg)), seed=np.array([seed]), fill=np.array([fill]),
               stream=np.array([tok0, kv_seed], np.int64), tokens=np.array(toks, np.int32),
               top_idx=np.stack(top_i), top_val=np.stack(top_v), margin=marg, maxabs=mx,
               full_at=np.array(FULL_AT, np.int32), full_logits=np.stack(full))
    np.savez_compressed(os.path.join(HERE, f"deep_long_{name}.npz"), **out)
    rel = marg / mx
    print(f"{name}: tokens {toks}", flush=True)
    print(f"{name}: margin/max min {rel.min():.4f} at step {int(rel.argmin())}; steps below 0.015: "
          f"{np.nonzero(rel <= 0.015)[0].tolist()}", flush=True)
    man = os.path.join(HERE, "manifest.json")
    with open(man) as f:
        manifest = json.load(f)
    manifest["files"][f"deep_long_{name}.npz"] = (
        f"full-depth oracle long greedy run (tests/golden/gen_deep_long.py, oracle/ti_oracle_deep.c), {what}: "
        f"engine seed {seed}, unit norms, (tok0, kv_seed) {(tok0, kv_seed)}: KV filled to {fill}, {N_LONG} greedy "
        f"steps; per step token, margin, max|logit|, top-{TOPK} logits; full logits at steps {list(FULL_AT)}")
    with open(man, "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"{name}: {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    o = Oracle()
    for n in (sys.argv[1:] or list(STREAMS)):
        make(n, o)
