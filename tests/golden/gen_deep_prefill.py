"""Full-depth PREFILL fixtures: a 120-token prompt from an empty cache, then
greedy decode, at the BASELINE models' real depth and width, from the full-depth oracle
(oracle/ti_oracle_deep.c, bit-identical to the pinned or_decode_step: tests/test_oracle_deep.py).

The oracle feeds the prompt one token per step (forward_pass over the prompt with the KV kept is
the same arithmetic row by row, inference_engine.cpp:1429-1491); the engine runs its first 119
tokens as ONE prefill chunk (tile GEMM at 119 rows, MFMA causal attention) and decodes from the
last prompt token.  Stored: the prompt, N_GEN greedy tokens, every generated step's fp32 logits.

The prompt is seeded random ids; its LAST token is searched (the 119-token prefix is computed once,
the cache rewound per candidate) until every generated step's top-2 margin exceeds MARGIN of
max|logit|, so the GPU test (TOL 5e-3) can assert every token.

    python tests/golden/gen_deep_prefill.py            # both configs (~10 min, 8 threads)
    python tests/golden/gen_deep_prefill.py llama2_7b
    TI_PF_PROMPT=640 python tests/golden/gen_deep_prefill.py   # deep_prefill640_*.npz

The 640-token variant is the prefill the benchmark times: with the engine's 512-row chunk limit the
first 639 prompt tokens run as a 512-row chunk then a 127-row chunk that attends over the first
chunk's K/V, both through the tile GEMM and the MFMA causal attention.
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
from pyoracle import Oracle, OracleDeepModel  # noqa: E402
from gen_deep import CONFIGS  # noqa: E402

N_PROMPT, N_GEN, MARGIN = int(os.environ.get("TI_PF_PROMPT", "120")), 3, 0.016
SUFFIX = "" if N_PROMPT == 120 else str(N_PROMPT)
PROMPT_SEED = {"llama2_7b": 7001, "llama3_8b": 7003}


def make(name: str, oracle: Oracle) -> None:
    what, cfg, seed, _streams = CONFIGS[name]
    t0 = time.time()
    m = OracleDeepModel(oracle, cfg, seed, 0.0)
    rng = np.random.RandomState(PROMPT_SEED[name])
    prompt = rng.randint(3, cfg["vocab"], size=N_PROMPT).tolist()
    for t in prompt[:-1]:
        m.step(t)
    print(f"{name}: prefix of {N_PROMPT - 1} tokens in {time.time() - t0:.0f} s", flush=True)
    cands = [prompt[-1]] + rng.randint(3, cfg["vocab"], size=200).tolist()
    for c in cands:
        m.set_len(N_PROMPT - 1)
        toks, lgs, t = [], [], c
        ok = True
        for _ in range(N_GEN):
            t, lg = m.step(t)
            srt = np.sort(lg)
            ok = ok and (srt[-1] - srt[-2]) > MARGIN * float(np.max(np.abs(lg)))
            toks.append(t)
            lgs.append(lg)
            if not ok:
                break
        if ok:
            prompt[-1] = c
            break
        print(f"  last token {c}: margin too small at step {len(toks) - 1}", flush=True)
    else:
        raise RuntimeError("no candidate last token with wide margins")
    lgs = np.stack(lgs)
    srt = np.sort(lgs, axis=1)
    out = dict(cfg=np.array(json.dumps(cfg)), seed=np.array([seed]), prompt=np.array(prompt, np.int32),
               tokens=np.array(toks, np.int32), logits=lgs.astype(np.float32),
               margin=(srt[:, -1] - srt[:, -2]).astype(np.float32))
    rel = out["margin"] / np.abs(lgs).max(axis=1)
    print(f"{name}: last prompt token {prompt[-1]}, tokens {toks}, margin/max {np.round(rel, 4).tolist()}", flush=True)
    m.close()
    np.savez_compressed(os.path.join(HERE, f"deep_prefill{SUFFIX}_{name}.npz"), **out)
    man = os.path.join(HERE, "manifest.json")
    with open(man) as f:
        manifest = json.load(f)
    manifest["files"][f"deep_prefill{SUFFIX}_{name}.npz"] = (
        f"full-depth oracle prefill + decode (tests/golden/gen_deep_prefill.py, oracle/ti_oracle_deep.c), {what}: "
        f"engine seed {seed}, unit norms, a {N_PROMPT}-token prompt (seeded, last token searched for margins "
        f"> {MARGIN} of max|logit|) from an empty cache, {N_GEN} greedy tokens with their logits")
    with open(man, "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"{name}: {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    o = Oracle()
    for n in (sys.argv[1:] or list(PROMPT_SEED)):
        make(n, o)
