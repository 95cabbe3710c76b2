"""Decode-engine parity (ti_engine.h) against the reference-composed decode (golden vectors
from the compiled reference) and the oracle.

Bars.  north_star: greedy token ids bit-exact; logits within 1e-2 relative.  The tests hold
the logits to TOL = 2e-3 * max|ref| per step, 5x tighter: the measured error is 5.6e-4 ..
8.4e-4 * max|ref| at every BASELINE config shape, one stream and 64 / 32 streams alike
(tools/parity_probe.py, round 2).  Greedy equality is then implied wherever the reference's
top-2 margin exceeds 2 * TOL; every checked step is asserted to have a margin above 3 * TOL
(seeds, prompts and streams chosen offline with tools/margin_search.py), and its token is
asserted equal -- no step is skipped (hard part 2).
"""
from __future__ import annotations

import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

f32 = np.float32
TOL = 2e-3


def engine_for(ti, cfg, max_batch=1, max_seq=None, splits=0):
    return ti.Engine(cfg["vocab"], cfg["hidden"], cfg["layers"], cfg["heads"], cfg["kv_heads"], cfg["head_dim"],
                     cfg["inter"], bits=cfg["bits"], max_seq=max_seq or cfg["max_seq"], max_batch=max_batch,
                     rope_theta=cfg["rope_theta"], eps=cfg["eps"], attn_splits=splits)


def margin(lg):
    s = np.sort(lg)
    return float(s[-1] - s[-2])


def assert_logits_close(got, ref):
    tol = TOL * float(np.max(np.abs(ref)))
    err = float(np.max(np.abs(got.astype(np.float64) - ref)))
    assert err <= tol, f"logit error {err} > {tol}"


def assert_greedy(got, ref, ref_logits, what=""):
    """Every step: the reference margin is wide (so the logits bound decides the token), and
    the tokens are equal."""
    assert len(got) == len(ref)
    for i, (g, r) in enumerate(zip(got, ref)):
        m, mx = margin(ref_logits[i]), float(np.max(np.abs(ref_logits[i])))
        assert m > 3 * TOL * mx, f"{what} step {i}: reference margin {m:.4g} <= 3 * TOL * {mx:.4g} (re-pick the seed)"
        assert g == r, f"{what} token {i}: gpu {g} ref {r} (margin {m})"


@pytest.mark.parametrize("name", ["mini_gqa_w4", "mini_hd128_w8"])
def test_engine_steps_match_reference_composed(ti, golden, name):
    d = golden(f"decode_{name}")
    cfg = json.loads(str(d["cfg"]))
    e = engine_for(ti, cfg)
    e.synth(int(d["seed"][0]), float(d["jitter"][0]))
    toks = d["tokens"].tolist()
    for pos in range(len(toks) - 1):
        lg = e.step([toks[pos]], [pos])[0]
        assert_logits_close(lg, d["logits"][pos])
    e.close()


@pytest.mark.parametrize("name", ["mini_gqa_w4", "mini_hd128_w8"])
def test_engine_greedy_tokens_match_reference(ti, golden, name):
    d = golden(f"decode_{name}")
    cfg = json.loads(str(d["cfg"]))
    prompt = d["prompt"].tolist()
    ref_new = d["tokens"].tolist()[len(prompt):]
    e = engine_for(ti, cfg)
    e.synth(int(d["seed"][0]), float(d["jitter"][0]))
    got = e.generate([prompt], len(ref_new))[0].tolist()
    assert_greedy(got, ref_new, d["logits"][len(prompt) - 1:], name)
    e.close()


def _oracle_tokens(oracle, cfg, seed, jitter, prompt, n_new, fill=0, kv_seed=0):
    from pyoracle import OracleModel
    m = OracleModel(oracle, cfg, seed, jitter)
    if fill:
        m.fill_kv(fill, kv_seed)
    out, logits, t = [], [], None
    for tok in prompt:
        t, lg = m.step(tok)
    out.append(t)
    logits.append(lg)
    for _ in range(n_new - 1):
        t, lg = m.step(out[-1])
        out.append(t)
        logits.append(lg)
    m.close()
    return out, logits


MID = dict(vocab=1024, hidden=512, layers=3, heads=8, kv_heads=1, head_dim=64, inter=768, rope_theta=10000.0,
           eps=1e-5, bits=4, group=128, max_seq=512)


def test_engine_gqa8_long_context_vs_oracle(ti, oracle):
    """GQA group 8, 300 synthetic cache slots, decode from position 300."""
    seed, jit, kv_seed, fill = 5, 0.1, 77, 300
    prompt = [3, 500, 1023]
    ref, ref_logits = _oracle_tokens(oracle, MID, seed, jit, prompt, 6, fill, kv_seed)
    e = engine_for(ti, MID)
    e.synth(seed, jit)
    e.fill_kv(0, fill, kv_seed)
    got, lg = e.generate([prompt], 6, start_pos=[fill], want_logits=True)
    assert_greedy(got[0].tolist(), ref, ref_logits)
    assert_logits_close(lg[0], ref_logits[-1])
    e.close()


def test_engine_batched_streams_independent(ti, oracle):
    """B streams with different prompts / start positions decode as B independent requests."""
    seed, jit = 9, 0.1
    prompts = [[1, 2, 3], [400], [7, 8, 9, 10, 11]]
    single = [_oracle_tokens(oracle, MID, seed, jit, p, 5) for p in prompts]
    e = engine_for(ti, MID, max_batch=4)
    e.synth(seed, jit)
    got = e.generate(prompts, 5)
    for b, (ref, ref_logits) in enumerate(single):
        assert_greedy(got[b].tolist(), ref, ref_logits, f"stream {b}")
    e.close()


def test_engine_replay_fixed_position(ti, oracle):
    """Benchmark replay: every step decodes at position kv_len-1 over a synthetic cache."""
    from pyoracle import OracleModel
    seed, jit, kv_seed, L, start = 13, 0.0, 21, 200, 42
    e = engine_for(ti, MID)
    e.synth(seed, jit)
    e.fill_kv(0, L - 1, kv_seed)
    e.replay_prepare(1, L, start)
    m = OracleModel(oracle, MID, seed, jit)
    tok = start
    for step in range(3):
        e.replay_run(1)
        e.sync()
        got = int(e.last_tokens(1)[0])
        m.fill_kv(L - 1, kv_seed)          # slot L-1 is rewritten every replay step
        ref, lg = m.step(tok)
        assert_greedy([got], [ref], [lg], f"replay step {step}")
        tok = got
    m.close()
    e.close()


# BASELINE config shapes, two layers each (parity probe + margin search, round 2)
CFG_7B = dict(vocab=32000, hidden=4096, layers=2, heads=32, kv_heads=32, head_dim=128, inter=11008,
              rope_theta=10000.0, eps=1e-5, bits=4, group=128, max_seq=2048)
CFG_TL = dict(vocab=32000, hidden=2048, layers=2, heads=32, kv_heads=4, head_dim=64, inter=5632,
              rope_theta=10000.0, eps=1e-5, bits=8, group=128, max_seq=2048)
CFG_L3 = dict(vocab=128256, hidden=4096, layers=2, heads=32, kv_heads=8, head_dim=128, inter=14336,
              rope_theta=500000.0, eps=1e-5, bits=4, group=128, max_seq=8192)


def _stream_params(seed, b, V):
    """Stream b of a synthetic batch: its first token and KV seed (tools/margin_search.py)."""
    return (seed * 7 + 13 * b) % V, 100 + b


def _full_shape_streams(ti, oracle, cfg, seed, B, checked, n_steps, slot_of=None):
    """B streams, each with its own synthetic cache of max_seq - n_steps slots and its own first
    token, decode n_steps tokens (the last at position max_seq - 1).  `checked` streams (logical
    indices; slot_of maps them to engine slots, default identity) are compared with the oracle:
    per-step logits through ti_engine_step (teacher-forced with the oracle's tokens) and the greedy
    tokens of ti_engine_generate (the device loop with argmax feedback)."""
    from pyoracle import OracleModel
    V, fill = cfg["vocab"], cfg["max_seq"] - n_steps
    slot_of = slot_of or (lambda b: b)
    m = OracleModel(oracle, cfg, seed, 0.0)
    ref = {}
    for b in checked:
        tok0, kvs = _stream_params(seed, b, V)
        m.fill_kv(fill, kvs)
        toks, lgs, t = [], [], tok0
        for _ in range(n_steps):
            t, lg = m.step(t)
            toks.append(t)
            lgs.append(lg)
        ref[b] = (tok0, toks, lgs)
    m.close()
    logical = {slot_of(b): b for b in checked}
    params = [_stream_params(seed, logical.get(s, s), V) for s in range(B)]
    e = engine_for(ti, cfg, max_batch=B)
    e.synth(seed, 0.0)
    for s in range(B):
        e.fill_kv(s, fill, params[s][1])
    feed = [p[0] for p in params]
    for step in range(n_steps):
        lg = e.step(feed, [fill + step] * B)
        for s, b in logical.items():
            assert_logits_close(lg[s], ref[b][2][step])
        feed = [int(t) for t in np.argmax(lg, axis=1)]
        for s, b in logical.items():
            feed[s] = ref[b][1][step]
    for s in range(B):
        e.fill_kv(s, fill, params[s][1])
    got = e.generate([[p[0]] for p in params], n_steps, start_pos=[fill] * B)
    e.close()
    for s, b in logical.items():
        assert_greedy(got[s].tolist(), ref[b][1], ref[b][2], f"stream {b}")


def test_engine_7b_shape_two_layers(ti, oracle):
    """BASELINE configs[2] shapes: Llama-2-7B layers (H 4096, I 11008, 32 heads x 128, vocab
    32000, INT4 g128), two layers, one stream decoding positions 2044..2047."""
    _full_shape_streams(ti, oracle, CFG_7B, 2025, 1, [1], 4, slot_of=lambda b: 0)


def test_engine_7b_64_streams(ti, oracle):
    """BASELINE configs[3] per GPU: 64 streams of Llama-2-7B shape (batch 512 over 8 replicas),
    each with its own 2044-slot cache and first token, four steps to position 2047: five streams
    spread over the batch (both 32-row GEMM chunks) against the oracle."""
    _full_shape_streams(ti, oracle, CFG_7B, 2025, 64, [1, 17, 35, 49, 63], 4)


def test_engine_7b_40_streams(ti, oracle):
    """40 streams of the 7B shape: the batched-rows kernel in three 16-row blocks for the narrow
    projections (O, down; whole XCD rows of column groups), the tile kernel for the wide ones
    (gate/up, lm_head: rows x N >= TI_GEMM_TILE_WIDE_MN); a stream in each row block against the
    oracle (the 64-stream test's streams, same caches and first tokens)."""
    _full_shape_streams(ti, oracle, CFG_7B, 2025, 40, [1, 17, 35], 4)


def test_engine_compat_plumbing_matches_reference_generate(ti, oracle, golden):
    """BASELINE config 1: the reference's own generate() on its benchmark model, exact tokens
    (fp32 bit-exact path + the reference sampler's tie order)."""
    d = golden("plumbing_generate")
    V, H, layers = 1000, 256, 4
    I = 4 * H
    e = ti.Engine(V, H, layers, 4, 4, 64, I, bits=16, max_seq=2048, max_batch=1, compat=True)
    # exact float32 evaluation of ((float)(i % 200) / 200.0f - 0.5f) * 0.02f (benchmark_inference.cpp:199-205)
    idx = np.arange(H * I)
    up = ((((idx % 200).astype(f32) / f32(200.0)) - f32(0.5)) * f32(0.02)).astype(f32).reshape(H, I)
    down = up.reshape(-1).reshape(I, H)
    lm = ((((np.arange(H * V) % 500).astype(f32) / f32(500.0)) - f32(0.5)) * f32(0.01)).astype(f32).reshape(H, V)
    for l in range(layers):
        e.set_tensor(ti.W_UP, l, up)
        e.set_tensor(ti.W_DOWN, l, down)
    e.set_tensor(ti.W_LM_HEAD, 0, lm)
    for i in range(3):
        prompt = d[f"prompt{i}"].tolist()
        toks = list(prompt)
        lg = e.compat_step((len(prompt) - 1) * H)
        for _ in range(20):
            t, _ = ti.sample_token(lg, 1.0, 1, 0.9, 0.5)
            toks.append(t)
            if t == 2:
                break
            lg = e.compat_step(0)
        assert toks == d[f"tokens{i}"].tolist()
        _, olog = oracle.plumbing_generate(V, H, layers, prompt, 1)
        lg0 = e.compat_step((len(prompt) - 1) * H)
        np.testing.assert_array_equal(lg0.view(np.uint32), olog.view(np.uint32))
    e.close()


def test_engine_tinyllama_int8_shape(ti, oracle):
    """BASELINE configs[1] shapes: TinyLlama-1.1B (H 2048, 32 q / 4 kv heads x 64, I 5632,
    vocab 32000) with INT8 g128 weights, two layers, one stream decoding positions 2044..2047."""
    _full_shape_streams(ti, oracle, CFG_TL, 1101, 1, [1], 4, slot_of=lambda b: 0)


def test_engine_llama3_8b_gqa_long_context_shape(ti, oracle):
    """BASELINE configs[4] shapes: Llama-3-8B (H 4096, 32 q / 8 kv heads x 128, I 14336,
    vocab 128256, rope theta 5e5) INT4 g128, two layers, one stream at positions 8189..8191."""
    _full_shape_streams(ti, oracle, CFG_L3, 808, 1, [8], 3, slot_of=lambda b: 0)


def test_engine_llama3_32_streams_8192(ti, oracle):
    """BASELINE configs[4]: 32 streams of Llama-3-8B GQA shape, each with its own 8189-slot
    cache (8192-token KV), three steps to position 8191: five streams against the oracle."""
    _full_shape_streams(ti, oracle, CFG_L3, 808, 32, [2, 8, 19, 24, 31], 3)


def test_engine_batch_beyond_one_gemm_chunk(ti, oracle):
    """20 streams (more than the 16 rows one GEMV launch takes): chunked M, every stream still
    an independent request."""
    seed, jit = 31, 0.1
    prompts = [[(7 * b + 1) % MID["vocab"], (11 * b + 5) % MID["vocab"]] for b in range(20)]
    e = engine_for(ti, MID, max_batch=20)
    e.synth(seed, jit)
    got = e.generate(prompts, 3)
    e.close()
    for b in (0, 7, 16, 19):
        ref, ref_logits = _oracle_tokens(oracle, MID, seed, jit, prompts[b], 3)
        assert_greedy(got[b].tolist(), ref, ref_logits, f"stream {b}")


def test_generate_stop_token_per_stream(ti):
    """ti_engine_set_stop (generate()'s EOS break, inference_engine.cpp:760-764) on two streams of one
    engine: stream 0 (prompt 1 17 42, seed 78) emits token 2 as its third token, stream 1 (prompt 7)
    not within 30.  With the stop set, stream 0's tokens end at its stop token (-1 after) and stream 1's
    are the tokens of the run without a stop; the loop runs every step (stream 1 never stops).  Stream
    0 alone stops after the first chunk of 4 steps (ti_engine_counters), not after 30."""
    cfg = dict(vocab=128, hidden=256, layers=2, heads=4, kv_heads=2, head_dim=64, inter=512, bits=4,
               max_seq=256, rope_theta=10000.0, eps=1e-5)
    e = engine_for(ti, cfg, max_batch=2)
    e.synth(78, 0.1)
    a, b, n = [1, 17, 42], [7], 30
    full = e.generate([a, b], n)
    full1 = e.generate([a], n)                           # (one stream: the M = 1 path)
    assert full[0][:3].tolist()[-1] == 2 and 2 not in full[0][:2].tolist(), full[0][:3]
    assert 2 not in full[1].tolist()
    d0, _ = e.counters()
    e.set_stop(2)
    got = e.generate([a, b], n)
    d1, _ = e.counters()
    assert got[0].tolist() == full[0][:3].tolist() + [-1] * (n - 3)
    assert got[1].tolist() == full[1].tolist()
    assert d1 - d0 == len(a) + n - 1 - (len(b) - 1)   # every step of the loop (prefill took len(b) - 1 = 0)
    one = e.generate([a], n)
    d2, _ = e.counters()
    e.close()
    assert one[0].tolist() == full1[0][:3].tolist() + [-1] * (n - 3)
    assert d2 - d1 == 4                                  # the first chunk covers the stop (3 tokens)


def test_generate_last_prompt_row_gives_first_token(ti):
    """Greedy streams whose prompts have one length: the last prompt token is a prefill row and the
    first token comes from the final rms_norm + lm_head on its hidden row (as the reference's
    forward_pass computes the last position's logits), not from a decode step.  Against the same
    prompt beside a shorter one (unequal lengths take the decode step for it): the same tokens,
    logits within the deep bar (5e-3 x max|logit|), and the step counts of ti_engine_counters."""
    cfg = dict(vocab=512, hidden=512, layers=4, heads=8, kv_heads=2, head_dim=64, inter=1024, bits=4,
               max_seq=512, rope_theta=10000.0, eps=1e-5)
    e = engine_for(ti, cfg, max_batch=2)
    e.synth(31, 0.1)
    e.set_prefill(64)                                     # 100-token prompts: chunks of 64 + 36 rows
    rng = np.random.RandomState(5)
    p1, p2 = ([int(t) for t in rng.randint(0, cfg["vocab"], size=100)] for _ in range(2))

    def run(prompts, k):
        d0, c0 = e.counters()
        out, lg = e.generate(prompts, k, want_logits=True)
        d1, c1 = e.counters()
        return out, lg, d1 - d0, c1 - c0

    for k in (1, 6):
        one, lg1, d, c = run([p1], k)
        assert (d, c) == (k - 1, 2)
        two, lg2, d, c = run([p1, p2], k)
        assert (d, c) == (k - 1, 4)
        # unequal lengths: stream 0 (the longer) through the decode step, which runs from the
        # shorter prompt's last token; its last step is stream 0's last prompt position
        ref1, rl1, d, c = run([p1, p2[:-1]], k)
        assert (d, c) == (k + 1, 4)
        ref2, rl2, _, _ = run([p2, p1[:-1]], k)
        assert one[0].tolist() == two[0].tolist() == ref1[0].tolist()
        assert two[1].tolist() == ref2[0].tolist()
        if k == 1:   # the last prompt position's logits, both ways
            for got, ref in ((lg1[0], rl1[0]), (lg2[0], rl1[0]), (lg2[1], rl2[0])):
                assert float(np.max(np.abs(got - ref))) <= 5e-3 * float(np.max(np.abs(ref)))
    e.close()


def test_generate_stop_at_the_prefill_token(ti):
    """The stop token as the first generated token, which the prefill's last row gives: the device
    loop runs no step at all (the reference breaks before its next forward pass), for max_new 1 and
    6, and the stop set with max_new 1 returns that token (ti_engine_counters)."""
    cfg = dict(vocab=512, hidden=512, layers=4, heads=8, kv_heads=2, head_dim=64, inter=1024, bits=4,
               max_seq=512, rope_theta=10000.0, eps=1e-5)
    e = engine_for(ti, cfg)
    e.synth(47, 0.1)
    e.set_prefill(64)
    p = [int(t) for t in np.random.RandomState(9).randint(0, cfg["vocab"], size=80)]
    ref = e.generate([p], 6)[0].tolist()
    e.set_stop(ref[1] if ref[1] != ref[0] else -1)         # a stop that is not the first token
    if ref[1] != ref[0]:
        assert e.generate([p], 6)[0].tolist() == ref[:2] + [-1] * 4
    e.set_stop(ref[0])
    for k in (1, 6):
        d0, _ = e.counters()
        got = e.generate([p], k)[0].tolist()
        d1, _ = e.counters()
        assert got == [ref[0]] + [-1] * (k - 1) and d1 == d0, (got, d1 - d0)
    e.close()
