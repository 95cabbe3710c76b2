"""Full-depth decode parity (VERDICT r2 'next' 1): the engine at the BASELINE configs' real
depth -- 32 layers of Llama-2-7B INT4 (configs[2], [3]), 22 of TinyLlama INT8 (configs[1]), 32
of Llama-3-8B GQA INT4 at an 8192-token cache (configs[4]) -- against the full-depth oracle
fixtures (tests/golden/gen_deep.py; oracle/ti_oracle_deep.c = the pinned or_decode_step).

Each checked stream: KV cache filled to max_seq - 3, then three decode steps, the last at the
bench's replay position max_seq - 1.  Per step the logits (teacher-forced through
ti_engine_step) are held to TOL * max|ref| and the greedy tokens of ti_engine_generate (device
argmax feedback) must equal the oracle's, each step's reference top-2 margin above 3 * TOL.
The batched cases put the fixture streams at the first and last slot of 64 (7B) / 32 (L3)
streams whose other slots hold their own caches and tokens.

TOL_DEEP = 5e-3 (north_star: 1e-2 relative).  The engine computes in fp16 activations and an fp16
KV cache with fp32 accumulation; the error grows with depth: 5.6-8.4e-4 * max|logit| at 2 layers
(test_gpu_engine.py, TOL 2e-3), 2.6e-3 at 32 layers of 7B (round 3, first run).

north_star's literal bound, "fp16 logits within 1e-2 relative", is also asserted per element on
the logits that decide the token: at every checked step the oracle's 16 largest logits, each
|y_i - r_i| / |r_i| <= TOL_ELEM = 1e-2 (the max-norm bound above covers the
rest of the vector, whose entries near zero make a per-element ratio meaningless).

Set TI_PARITY_LOG=<file> to append each checked stream's measured error (JSON lines)."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from test_gpu_engine import engine_for, margin

pytestmark = pytest.mark.gpu

TOL = TOL_DEEP = 5e-3
TOL_ELEM = 1e-2   # north_star: per element, relative, on the oracle's top-16 logits of each step


def top16_rel(got, ref):
    """max over the oracle's 16 largest logits of |got_i - ref_i| / |ref_i|."""
    ref = np.asarray(ref, np.float64)
    idx = np.argpartition(ref, -16)[-16:]
    return float(np.max(np.abs(np.asarray(got, np.float64)[idx] - ref[idx]) / np.abs(ref[idx])))


def assert_greedy(got, ref, ref_logits, what=""):
    """Every step: the reference margin exceeds 3 * TOL * max|logit| (so the logits bound decides
    the token), and the tokens are equal."""
    assert len(got) == len(ref)
    for i, (g, r) in enumerate(zip(got, ref)):
        m, mx = margin(ref_logits[i]), float(np.max(np.abs(ref_logits[i])))
        assert m > 3 * TOL * mx, f"{what} step {i}: reference margin {m:.4g} <= 3 * TOL * {mx:.4g} (re-pick)"
        assert g == r, f"{what} token {i}: gpu {g} ref {r} (margin {m})"


def _fixture(golden, name):
    d = golden(f"deep_{name}")
    cfg = json.loads(str(d["cfg"]))
    streams = [tuple(int(v) for v in s) for s in d["streams"]]
    ref = [(d[f"tokens{i}"].tolist(), d[f"logits{i}"]) for i in range(len(streams))]
    return cfg, int(d["seed"][0]), int(d["fill"][0]), streams, ref


def _log(rec):
    path = os.environ.get("TI_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def _run(ti, golden, name, B, slots, which=None):
    """slots[i] = engine slot of fixture stream which[i] (default i); the other slots get their own
    (tok0, kv seed)."""
    cfg, seed, fill, streams, ref = _fixture(golden, name)
    which = which or list(range(len(slots)))
    streams, ref = [streams[w] for w in which], [ref[w] for w in which]
    V = cfg["vocab"]
    params = [((seed * 7 + 13 * s) % V, 1000 + s) for s in range(B)]
    for i, s in enumerate(slots):
        params[s] = streams[i]
    e = engine_for(ti, cfg, max_batch=B)
    e.synth(seed, 0.0)
    for s in range(B):
        e.fill_kv(s, fill, params[s][1])
    n = len(ref[0][0])
    feed = [p[0] for p in params]
    worst, worst16 = {}, {}
    for step in range(n):
        lg = e.step(feed, [fill + step] * B)
        feed = [int(t) for t in np.argmax(lg, axis=1)]
        for i, s in enumerate(slots):
            r = ref[i][1][step].astype(np.float64)
            mx = float(np.max(np.abs(r)))
            err = float(np.max(np.abs(lg[s].astype(np.float64) - r)))
            worst[i] = max(worst.get(i, 0.0), err / mx)
            worst16[i] = max(worst16.get(i, 0.0), top16_rel(lg[s], r))
            feed[s] = ref[i][0][step]
    for i, s in enumerate(slots):
        _log(dict(config=name, streams=B, slot=s, layers=cfg["layers"], max_rel_err=worst[i], tol=TOL,
                  top16_max_rel_err=worst16[i], tol_elem=TOL_ELEM))
        assert worst[i] <= TOL, f"{name} stream {i}: logit error {worst[i]:.4g} * max|logit| > {TOL}"
        assert worst16[i] <= TOL_ELEM, f"{name} stream {i}: top-16 logit relative error {worst16[i]:.4g} > {TOL_ELEM}"
    for s in range(B):
        e.fill_kv(s, fill, params[s][1])
    got = e.generate([[p[0]] for p in params], n, start_pos=[fill] * B)
    e.close()
    for i, s in enumerate(slots):
        assert_greedy(got[s].tolist(), ref[i][0], ref[i][1], f"{name} stream {i}")


def test_deep_llama2_7b_one_stream(ti, golden):
    """configs[2]: the bench's model at full depth, one stream, positions 2045..2047."""
    _run(ti, golden, "llama2_7b", 1, [0])


def test_deep_llama2_7b_second_stream(ti, golden):
    """The second fixture stream of configs[2] alone (its own cache and first token)."""
    _run(ti, golden, "llama2_7b", 1, [0], which=[1])


def test_deep_llama2_7b_64_streams(ti, golden):
    """configs[3] per GPU: 64 streams at full depth; fixture streams in slots 1 and 63 (both
    32-row halves of the batched GEMMs)."""
    _run(ti, golden, "llama2_7b", 64, [1, 63])


def test_deep_tinyllama_one_stream(ti, golden):
    """configs[1]: 22 layers of TinyLlama INT8 (GQA 8, hd 64), one stream."""
    _run(ti, golden, "tinyllama_1b", 1, [0])


def test_deep_llama3_8b_one_stream(ti, golden):
    """configs[4] shape, one stream at the 8192-token cache: 32 layers, GQA 4, vocab 128256."""
    _run(ti, golden, "llama3_8b", 1, [0])


def test_deep_llama3_8b_32_streams(ti, golden):
    """configs[4]: 32 streams of 8192-token caches at full depth; fixture streams in slots 8 and 31."""
    _run(ti, golden, "llama3_8b", 32, [8, 31])


@pytest.mark.parametrize("name", ["llama2_7b", "tinyllama_1b", "llama3_8b"])
def test_deep_bench_replay(ti, golden, name):
    """The path bench.py times (ti_engine_replay_*): cache filled to max_seq - 1, every step at
    position max_seq - 1 fed the previous step's device argmax, two steps against the oracle."""
    d = golden(f"deep_{name}")
    cfg, seed, _fill, streams, _ref = _fixture(golden, name)
    tok0, kv_seed = (int(v) for v in d["replay"])
    L = cfg["max_seq"]
    e = engine_for(ti, cfg, max_batch=1)
    e.synth(seed, 0.0)
    e.fill_kv(0, L - 1, kv_seed)
    e.replay_prepare(1, L, tok0)
    got = []
    for _ in range(2):
        e.replay_run(1)
        e.sync()
        got.append(int(e.last_tokens(1)[0]))
    e.close()
    assert_greedy(got, d["replay_tokens"].tolist(), d["replay_logits"], f"{name} replay")


@pytest.mark.parametrize("name", ["llama2_7b", "llama3_8b"])
def test_deep_prefill_then_decode(ti, golden, name):
    """prefill at full width and depth.  A 120-token prompt from an empty cache
    (tests/golden/gen_deep_prefill.py): the engine runs the 120 tokens as ONE prefill chunk -- the
    tile GEMM at 120 rows and the MFMA causal attention, at every one of the 32 layers; the first
    token's logits from the last row's lm_head, the KV they write then read by the decode steps --
    and decodes 2 more greedy tokens (reference forward_pass + forward_pass_incremental,
    inference_engine.cpp:1429-1552).  Every
    generated step's logits within TOL_DEEP * max|logit| of the full-depth oracle (which feeds the
    prompt token by token), and every token equal."""
    d = golden(f"deep_prefill_{name}")
    cfg = json.loads(str(d["cfg"]))
    prompt, ref, ref_lg = d["prompt"].tolist(), d["tokens"].tolist(), d["logits"]
    e = engine_for(ti, cfg, max_batch=1)
    e.synth(int(d["seed"][0]), 0.0)
    worst = worst16 = 0.0
    for n in range(1, len(ref) + 1):   # logits of generated step n - 1 (each call prefills again)
        got, lg = e.generate([prompt], n, want_logits=True)
        r = ref_lg[n - 1].astype(np.float64)
        worst = max(worst, float(np.max(np.abs(lg[0].astype(np.float64) - r))) / float(np.max(np.abs(r))))
        worst16 = max(worst16, top16_rel(lg[0], r))
    e.close()
    _log(dict(config=name, case="prefill120+decode3", layers=cfg["layers"], max_rel_err=worst, tol=TOL,
              top16_max_rel_err=worst16, tol_elem=TOL_ELEM))
    assert worst <= TOL, f"{name}: logit error {worst:.4g} * max|logit| > {TOL}"
    assert worst16 <= TOL_ELEM, f"{name}: top-16 logit relative error {worst16:.4g} > {TOL_ELEM}"
    assert_greedy(got[0].tolist(), ref, ref_lg, f"{name} prefill")


@pytest.mark.parametrize("rows", [512, 1024])
@pytest.mark.parametrize("name", ["llama2_7b", "llama3_8b"])
def test_deep_prefill_512_row_chunks(ti, golden, name, rows):
    """prefill at the chunk size it is timed at.  A 640-token prompt
    (tests/golden/gen_deep_prefill.py, TI_PF_PROMPT=640) with the engine's chunk limit at 512 rows:
    the prompt runs as a 512-row chunk (the 7B / Llama-3 tile plans at 512 rows) and then a 128-row
    chunk whose causal attention reads the first chunk's K/V, at all 32 layers, and whose last row
    gives the first token; then 2 greedy decode steps.  Logits within TOL_DEEP * max|logit| of the oracle at every generated step, every
    token equal, and the engine's counters show the two prompt chunks per call.  With the int4
    default limit (1024 rows) the whole prompt is one 640-row chunk."""
    d = golden(f"deep_prefill640_{name}")
    cfg = json.loads(str(d["cfg"]))
    prompt, ref, ref_lg = d["prompt"].tolist(), d["tokens"].tolist(), d["logits"]
    assert len(prompt) == 640
    e = engine_for(ti, cfg, max_batch=1)
    e.synth(int(d["seed"][0]), 0.0)
    e.set_prefill(rows)
    worst = worst16 = 0.0
    for n in range(1, len(ref) + 1):
        _, c0 = e.counters()
        got, lg = e.generate([prompt], n, want_logits=True)
        assert e.counters()[1] - c0 == (2 if rows == 512 else 1)   # 512 + 128 prompt rows, or 640
        r = ref_lg[n - 1].astype(np.float64)
        worst = max(worst, float(np.max(np.abs(lg[0].astype(np.float64) - r))) / float(np.max(np.abs(r))))
        worst16 = max(worst16, top16_rel(lg[0], r))
    e.close()
    _log(dict(config=name, case=f"prefill640(chunks of {rows})+decode3", layers=cfg["layers"], max_rel_err=worst, tol=TOL,
              top16_max_rel_err=worst16, tol_elem=TOL_ELEM))
    assert worst <= TOL, f"{name}: logit error {worst:.4g} * max|logit| > {TOL}"
    assert worst16 <= TOL_ELEM, f"{name}: top-16 logit relative error {worst16:.4g} > {TOL_ELEM}"
    assert_greedy(got[0].tolist(), ref, ref_lg, f"{name} prefill 512-row chunks")


def _long_run(ti, golden, name, B, slot):
    """VERDICT r3 weak 1 (drift over a longer greedy run at full depth): 64 decode steps of one
    stream (tests/golden/gen_deep_long.py), the last at max_seq - 1, every step attending over the
    K/V rows the engine itself wrote on the earlier steps.

    Teacher-forced (ti_engine_step fed the oracle's tokens): at every step the oracle's top-16
    logits within TOL * max|logit|, the full logit vector at the fixture's full_at steps, and the
    argmax equal wherever the reference margin exceeds 3 * TOL * max|logit|.  Free-running
    (ti_engine_generate, device argmax feedback): the tokens equal the oracle's up to the first
    step whose margin is within 3 * TOL (a near-tie either side may take; the runs part there);
    a mismatch at any wider-margin step fails.  Logged: the per-step error curve."""
    d = golden(f"deep_long_{name}")
    cfg = json.loads(str(d["cfg"]))
    seed, fill = int(d["seed"][0]), int(d["fill"][0])
    tok0, kv_seed = (int(v) for v in d["stream"])
    ref, top_i, top_v = d["tokens"].tolist(), d["top_idx"], d["top_val"].astype(np.float64)
    marg, mx = d["margin"].astype(np.float64), d["maxabs"].astype(np.float64)
    full = {int(s): d["full_logits"][i].astype(np.float64) for i, s in enumerate(d["full_at"])}
    n, V = len(ref), cfg["vocab"]
    params = [((seed * 7 + 13 * s) % V, 1000 + s) for s in range(B)]
    params[slot] = (tok0, kv_seed)
    e = engine_for(ti, cfg, max_batch=B)
    e.synth(seed, 0.0)
    for s in range(B):
        e.fill_kv(s, fill, params[s][1])
    feed = [p[0] for p in params]
    curve, curve16, bad = [], [], []
    for step in range(n):
        lg = e.step(feed, [fill + step] * B)
        feed = [int(t) for t in np.argmax(lg, axis=1)]
        g = lg[slot].astype(np.float64)
        err = float(np.max(np.abs(g[top_i[step]] - top_v[step])))
        curve16.append(float(np.max(np.abs(g[top_i[step]] - top_v[step]) / np.abs(top_v[step]))))
        if curve16[-1] > TOL_ELEM:
            bad.append(f"step {step}: top-16 logit relative error {curve16[-1]:.4g} > {TOL_ELEM}")
        if step in full:
            err = max(err, float(np.max(np.abs(g - full[step]))))
        curve.append(err / mx[step])
        if curve[-1] > TOL:
            bad.append(f"step {step}: logit error {curve[-1]:.4g} * max|logit|")
        if marg[step] > 3 * TOL * mx[step] and int(np.argmax(g)) != ref[step]:
            bad.append(f"step {step}: argmax {int(np.argmax(g))} != {ref[step]} (margin {marg[step]:.4g})")
        feed[slot] = ref[step]
    for s in range(B):
        e.fill_kv(s, fill, params[s][1])
    got = e.generate([[p[0]] for p in params], n, start_pos=[fill] * B)[slot].tolist()
    e.close()
    matched = 0
    for step in range(n):
        if got[step] != ref[step]:
            if marg[step] > 3 * TOL * mx[step]:
                bad.append(f"generate step {step}: token {got[step]} != {ref[step]} (margin {marg[step]:.4g})")
            break
        matched += 1
    c = np.array(curve)
    _log(dict(config=name, case=f"long{n}", streams=B, slot=slot, layers=cfg["layers"], max_rel_err=float(c.max()),
              err_by_16_steps=[round(float(c[i:i + 16].max()), 6) for i in range(0, n, 16)],
              generate_matched=matched, first_near_tie=int(np.argmax(marg <= 3 * TOL * mx)), tol=TOL,
              top16_max_rel_err=float(max(curve16)), tol_elem=TOL_ELEM))
    assert not bad, f"{name} long run: " + "; ".join(bad)


def test_deep_long_llama2_7b(ti, golden):
    """configs[2]: 64 greedy steps of Llama-2-7B INT4 at full depth, positions 1984..2047."""
    _long_run(ti, golden, "llama2_7b", 1, 0)


def test_deep_long_llama2_7b_64_streams(ti, golden):
    """configs[3]: the same 64-step stream in slot 63 of 64 (the batched GEMMs' second half)."""
    _long_run(ti, golden, "llama2_7b", 64, 63)


def test_deep_long_tinyllama(ti, golden):
    """configs[1]: 64 greedy steps of TinyLlama INT8 at full depth, positions 1984..2047."""
    _long_run(ti, golden, "tinyllama_1b", 1, 0)
