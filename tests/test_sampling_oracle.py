"""Sampling parity on the CPU.

1. The oracle's sampler (oracle/ti_oracle_sample.cpp, a restatement of sample_next_token,
   inference_engine.cpp:1554-1673) is pinned to the REFERENCE: tests/golden/sample_plumbing.npz
   holds the (token, log-prob) pairs the compiled reference's own generate(include_logprobs)
   sampled on the plumbing model under eight (temperature, top-k, top-p) settings.  Its draws
   come from a clock-seeded mt19937 (:470-473) and are not observable, so each pair is checked
   through the interval of draws that select it: the token carries probability in the
   oracle's distribution, and a draw inside its interval makes the oracle return that token
   with a log-prob bit-identical to the reference's.  The plumbing lm_head repeats every 500
   columns, so every logit is tied with another one: top-k = 2, 3, 7, 9 cut through ties,
   resolved by libstdc++'s std::sort exactly as in the reference.
2. The product's host sampler (ti_sample_token, csrc/host/sampling.cpp) returns the oracle's
   token and bit-identical log-prob over a grid of logits (random, tied), settings and draws.
The device sampler is held to the oracle in tests/test_gpu_sample.py.
"""
from __future__ import annotations

import numpy as np
import pytest

f32 = np.float32
PROMPT = [1, 15, 25, 35]


@pytest.fixture(scope="module")
def plumbing_logits(oracle):
    """Logits the reference's plumbing generate() samples from at steps 0 and >= 1 (its
    placeholder embedding makes them independent of the sampled tokens; step >= 1 rows are
    all the same, inference_engine.cpp:1509-1512)."""
    return [oracle.plumbing_generate(1000, 256, 4, PROMPT, s + 1)[1] for s in range(2)]


def _u_for(probs, tok):
    """A draw that selects `tok` in the reference's ascending scan (u <= running sum)."""
    cum = np.cumsum(probs, dtype=f32)
    return float(cum[tok])


def test_oracle_sampler_pinned_to_reference_generate(oracle, golden, plumbing_logits):
    d = golden("sample_plumbing")
    checked = 0
    for i in range(int(d["n"][0])):
        T, k, p = (float(x) for x in d[f"cfg{i}"])
        k = int(k)
        toks, lps = d[f"tokens{i}"][len(PROMPT):], d[f"logprobs{i}"]
        assert len(toks) == len(lps) and len(toks) >= 1
        for s, (tok, lp) in enumerate(zip(toks.tolist(), lps)):
            lg = plumbing_logits[min(s, 1)]
            probs = oracle.sample_probs(lg, T, k, p)
            assert probs[tok] > 0, (i, s, tok)
            t, olp = oracle.sample_token(lg, T, k, p, _u_for(probs, tok))
            assert t == tok, (i, s, t, tok)
            assert np.float32(olp).view(np.uint32) == np.float32(lp).view(np.uint32), (i, s, olp, lp)
            checked += 1
    assert checked >= 80


def _grid_logits(plumbing_logits):
    rng = np.random.RandomState(2024)
    sets = [(rng.standard_normal(1000) * 3).astype(f32), (rng.standard_normal(32000) * 2).astype(f32),
            np.round(rng.standard_normal(4000) * 4).astype(f32) * f32(0.5)]     # many exact ties
    return sets + [np.asarray(x, f32) for x in plumbing_logits]


SETTINGS = [(1.0, 1, 0.9), (1.0, 50, 0.9), (0.7, 40, 0.9), (1.3, 0, 0.95), (1.0, 3, 1.0), (0.5, 1000, 0.5),
            (2.0, 7, 0.99), (0.0, 8, 0.5), (1.0, 200, 0.0), (0.8, 2000, 1.0), (1.0, 0, 1.0)]


def test_host_sampler_matches_oracle(ti_host, oracle, plumbing_logits):
    rng = np.random.RandomState(7)
    for lg in _grid_logits(plumbing_logits):
        for T, k, p in SETTINGS:
            kk = min(k, lg.size)
            probs = oracle.sample_probs(lg, T, kk, p)
            cum = np.cumsum(probs, dtype=f32)
            nz = np.flatnonzero(probs)
            draws = [0.0, 1.0, 0.5] + rng.uniform(0, 1, 6).tolist() + [float(cum[j]) for j in nz[:3]]
            for u in draws:
                want_t, want_lp = oracle.sample_token(lg, T, kk, p, u)
                got_t, got_lp = ti_host.sample_token(lg, T, kk, p, u)
                assert got_t == want_t, (T, k, p, u, got_t, want_t)
                assert np.float32(got_lp).view(np.uint32) == np.float32(want_lp).view(np.uint32), (T, k, p, u)


def test_reference_tie_order_is_exercised(oracle, golden, plumbing_logits):
    """The top-3 cut of the plumbing logits falls inside a tied pair: only one of the two
    equal logits survives, which one is decided by the reference's std::sort."""
    lg = plumbing_logits[1]
    probs = oracle.sample_probs(lg, 1.0, 3, 1.0)
    third = np.sort(lg)[-3]
    tied = np.flatnonzero(lg == third)
    assert tied.size == 2 and int(np.count_nonzero(probs[tied])) == 1
