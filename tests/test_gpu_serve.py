"""Continuous batching (ti_engine_serve): requests through max_batch stream slots, queued
requests admitted (prefilled) into slots that finished, the rest continuing at their own
positions.

Each request must decode as if it ran alone: against the oracle's reference-composed decode
of that prompt (greedy equality on every step, prompts chosen with every reference margin
above 3 x the logits tolerance, as in test_gpu_engine.py), and -- since the batched kernels compute every row from its own inputs -- bit for bit
the same whatever the chunking of the device loop (which changes which requests share a
chunk and when slots turn over).  An EOS ends a request early and frees its slot.
"""
from __future__ import annotations

import numpy as np
import pytest

from test_gpu_engine import MID, _oracle_tokens, assert_greedy, engine_for

pytestmark = pytest.mark.gpu

PROMPTS = [[1, 2, 3], [400], [7, 8, 9, 10, 11], [5, 7], [100, 200, 300, 400, 500, 600, 700], [12], [42, 43, 44]]


def test_serve_requests_decode_independently(ti, oracle):
    seed, jit, new = 9, 0.1, 6
    e = engine_for(ti, MID, max_batch=3)
    e.synth(seed, jit)
    got = e.serve(PROMPTS, new, eos=-1, chunk=4)
    got7 = e.serve(PROMPTS, new, eos=-1, chunk=7)
    got1 = e.serve(PROMPTS, new, eos=-1, chunk=1)
    e.close()
    assert got == got7 == got1
    for p, g in zip(PROMPTS, got):
        assert len(g) == new
        ref, ref_logits = _oracle_tokens(oracle, MID, seed, jit, p, new)
        assert_greedy(g, ref, ref_logits, f"request {p}")


def test_serve_eos_frees_the_slot(ti):
    seed, jit, new = 9, 0.1, 6
    e = engine_for(ti, MID, max_batch=2)
    e.synth(seed, jit)
    full = e.serve(PROMPTS, new, eos=-1, chunk=3)
    eos = full[0][1]                       # request 0 stops after its second token
    cut = e.serve(PROMPTS, new, eos=eos, chunk=3)
    e.close()
    for f, c in zip(full, cut):
        want = f[: f.index(eos) + 1] if eos in f else f
        assert c == want
