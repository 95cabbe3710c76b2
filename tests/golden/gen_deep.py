"""Full-depth decode fixtures (VERDICT r2 'next' 1): the BASELINE configs at their real depth,
width and context, from the full-depth oracle (oracle/ti_oracle_deep.c, bit-identical to the
pinned or_decode_step: tests/test_oracle_deep.py).

Per config and stream: the synthetic model (engine seed, unit norms as bench.py), the stream's
KV cache filled with synthetic fp16 rows up to max_seq - 3 (kv seed), then three greedy decode
steps from token tok0 at positions max_seq - 3 .. max_seq - 1 (the last one is the bench's
replay position).  Stored: the tokens, every step's fp32 logits, and the top-2 margins.

    python tests/golden/gen_deep.py            # all configs (~3 min, 8 threads, <= 12 GB)
    python tests/golden/gen_deep.py llama2_7b  # one config
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
from pyoracle import Oracle, OracleDeepModel  # noqa: E402

N_STEPS = 3

# name -> (BASELINE config, model, engine seed, streams [(tok0, kv_seed)]); REPLAY[name] = (tok0, kv_seed)
# of the bench-replay case.  Stream parameters were picked (offline, this oracle) so that every
# step's top-2 margin exceeds 1.5 % of max|logit| (the GPU tests need 3 x TOL_DEEP).
CONFIGS = {
    "llama2_7b": ("configs[2] / configs[3]: Llama-2-7B INT4 g128, KV 2048",
                  dict(vocab=32000, hidden=4096, layers=32, heads=32, kv_heads=32, head_dim=128, inter=11008,
                       rope_theta=10000.0, eps=1e-5, bits=4, group=128, max_seq=2048),
                  2025, [(4321, 100), (17, 163)]),
    "tinyllama_1b": ("configs[1]: TinyLlama-1.1B INT8 g128, KV 2048",
                     dict(vocab=32000, hidden=2048, layers=22, heads=32, kv_heads=4, head_dim=64, inter=5632,
                          rope_theta=10000.0, eps=1e-5, bits=8, group=128, max_seq=2048),
                     1101, [(2718, 101)]),
    "llama3_8b": ("configs[4]: Llama-3-8B GQA INT4 g128, KV 8192",
                  dict(vocab=128256, hidden=4096, layers=32, heads=32, kv_heads=8, head_dim=128, inter=14336,
                       rope_theta=500000.0, eps=1e-5, bits=4, group=128, max_seq=8192),
                  808, [(90001, 108), (31337, 131)]),
}


REPLAY = {"llama2_7b": (4321, 100), "tinyllama_1b": (1000, 101), "llama3_8b": (4242, 108)}


def make(name: str, oracle: Oracle) -> None:
    what, cfg, seed, streams = CONFIGS[name]
    t0 = time.time()
    m = OracleDeepModel(oracle, cfg, seed, 0.0)
    fill = cfg["max_seq"] - N_STEPS
    out = dict(cfg=np.array(json.dumps(cfg)), seed=np.array([seed]), fill=np.array([fill]),
               streams=np.array(streams, np.int64))
    for i, (tok0, kv_seed) in enumerate(streams):
        m.fill_kv(fill, kv_seed)
        toks, lgs, t = [], [], tok0
        for _ in range(N_STEPS):
            t, lg = m.step(t)
            toks.append(t)
            lgs.append(lg)
        lgs = np.stack(lgs)
        srt = np.sort(lgs, axis=1)
        out[f"tokens{i}"] = np.array(toks, np.int32)
        out[f"logits{i}"] = lgs.astype(np.float32)
        out[f"margin{i}"] = (srt[:, -1] - srt[:, -2]).astype(np.float32)
        rel = out[f"margin{i}"] / np.abs(lgs).max(axis=1)
        print(f"{name} stream {i}: tokens {toks} margin/max {np.round(rel, 4).tolist()}", flush=True)
    # bench replay (bench.py / ti_engine_replay_*): cache filled to max_seq - 1 with stream 0's kv
    # seed, every step at position max_seq - 1 (slot max_seq - 1 rewritten), fed the previous argmax
    tok0, kv_seed = REPLAY[name]
    out["replay"] = np.array([tok0, kv_seed], np.int64)
    toks, lgs, t = [], [], tok0
    for _ in range(2):
        m.fill_kv(cfg["max_seq"] - 1, kv_seed)
        t, lg = m.step(t)
        toks.append(t)
        lgs.append(lg)
    out["replay_tokens"] = np.array(toks, np.int32)
    out["replay_logits"] = np.stack(lgs).astype(np.float32)
    print(f"{name} replay: tokens {toks}", flush=True)
    m.close()
    np.savez_compressed(os.path.join(HERE, f"deep_{name}.npz"), **out)
    man = os.path.join(HERE, "manifest.json")
    with open(man) as f:
        manifest = json.load(f)
    manifest["files"][f"deep_{name}.npz"] = (
        f"full-depth oracle decode (tests/golden/gen_deep.py, oracle/ti_oracle_deep.c), {what}: engine seed {seed}, "
        f"unit norms, per stream (tok0, kv_seed) {streams}: KV filled to {fill}, {N_STEPS} greedy steps; "
        f"replay_*: (tok0, kv_seed) {REPLAY[name]} replayed twice at position {cfg['max_seq'] - 1} over a "
        f"{cfg['max_seq'] - 1}-slot fill")
    with open(man, "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"{name}: {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    o = Oracle()
    for n in (sys.argv[1:] or list(CONFIGS)):
        make(n, o)
