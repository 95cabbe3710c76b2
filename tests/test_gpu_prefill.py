"""Prefill (reference forward_pass, inference_engine.cpp:1429-1491, keeping the KV): a prompt's
tokens run as rows of the batched GEMMs with causal attention over the stream's own cache
(ti_engine_set_prefill), instead of one token per decode step.

Bars as in test_gpu_engine.py: logits within TOL x max|logit| of the oracle's
reference-composed decode, greedy tokens equal on every step (prompts chosen so that every
reference margin exceeds 3 x TOL); prefill and token-by-token feeding of the same prompt agree to
the same bar (they differ only in fp32 summation order and fp16 rounding of the KV)."""
from __future__ import annotations

import numpy as np
import pytest

from test_gpu_engine import MID, TOL, _oracle_tokens, assert_greedy, assert_logits_close, engine_for

pytestmark = pytest.mark.gpu

MID8 = dict(MID, kv_heads=4, head_dim=128, heads=4, bits=8)


@pytest.mark.parametrize("cfg", [MID, MID8], ids=["gqa8_w4", "mha_hd128_w8"])
def test_prefill_long_prompt_vs_oracle(ti, oracle, cfg):
    """70-token prompt: 3 prefill chunks (32, 32, 5 rows) + the decode loop."""
    seed, jit = 13, 0.1
    rng = np.random.RandomState(3)
    prompt = rng.randint(0, cfg["vocab"], size=70).tolist()
    ref, ref_logits = _oracle_tokens(oracle, cfg, seed, jit, prompt, 4)
    e = engine_for(ti, cfg)
    e.synth(seed, jit)
    got, lg = e.generate([prompt], 4, want_logits=True)
    assert_greedy(got[0].tolist(), ref, ref_logits)
    assert_logits_close(lg[0], ref_logits[-1])
    e.close()


def test_prefill_matches_token_by_token(ti, oracle):
    """Same engine, same prompt: prefill on vs off (and several streams, ragged prompts), both
    against the oracle."""
    seed, jit = 17, 0.1
    rng = np.random.RandomState(8)
    prompts = [rng.randint(0, MID["vocab"], size=n).tolist() for n in (41, 45, 64)]
    outs = []
    for rows in (ti.GEMM_MAX_ROWS, 0):
        e = engine_for(ti, MID, max_batch=3)
        e.synth(seed, jit)
        e.set_prefill(rows)
        outs.append(e.generate(prompts, 5, want_logits=True))
        e.close()
    (tp, lp), (tt, lt) = outs
    for b in range(3):
        ref, ref_logits = _oracle_tokens(oracle, MID, seed, jit, prompts[b], 5)
        assert_greedy(tp[b].tolist(), ref, ref_logits, f"prefill stream {b}")
        assert_greedy(tt[b].tolist(), ref, ref_logits, f"token-by-token stream {b}")
        # the device loop runs every stream for the longest prompt's step count, so the last
        # logits are the oracle's final step for the longest prompt only; the two feeds agree
        assert float(np.max(np.abs(lp[b].astype(np.float64) - lt[b]))) <= 2 * TOL * float(np.max(np.abs(lt[b])))
    assert_logits_close(lp[2], ref_logits[-1])
    assert_logits_close(lt[2], ref_logits[-1])


def test_prefill_start_pos_and_cache_contents(ti, oracle):
    """Prefill from a non-zero start position over a synthetic cache prefix."""
    seed, jit, kv_seed, fill = 5, 0.1, 77, 100
    rng = np.random.RandomState(7)
    prompt = rng.randint(0, MID["vocab"], size=37).tolist()
    ref, ref_logits = _oracle_tokens(oracle, MID, seed, jit, prompt, 3, fill, kv_seed)
    e = engine_for(ti, MID)
    e.synth(seed, jit)
    e.fill_kv(0, fill, kv_seed)
    got, lg = e.generate([prompt], 3, start_pos=[fill], want_logits=True)
    assert_greedy(got[0].tolist(), ref, ref_logits)
    assert_logits_close(lg[0], ref_logits[-1])
    e.close()


@pytest.mark.parametrize("rows,n", [(256, 300), (None, 300), (None, 1000)])
def test_prefill_tile_chunk_vs_oracle(ti, oracle, rows, n):
    """A 300-token prompt: with 256-row chunks, one through the LDS-tiled GEMM (ti_gemm_packed_rows
    says row-major there) and a 43-row chunk through the batched-rows kernel (packed); with the
    default chunk (TI_GEMM_MAX_ROWS) the prompt runs as one 299-row tile chunk, and a 1000-token
    prompt as one 999-row chunk (tile GEMM and MFMA attention at their largest row counts)."""
    cfg = dict(MID, max_seq=1024)
    seed, jit = 21, 0.1
    prompt = np.random.RandomState(9 if n == 300 else 10).randint(0, cfg["vocab"], size=n).tolist()   # wide margins
    ref, ref_logits = _oracle_tokens(oracle, cfg, seed, jit, prompt, 3)
    e = engine_for(ti, cfg)
    e.synth(seed, jit)
    if rows:
        e.set_prefill(rows)
    got, lg = e.generate([prompt], 3, want_logits=True)
    assert_greedy(got[0].tolist(), ref, ref_logits)
    assert_logits_close(lg[0], ref_logits[-1])
    e.close()
