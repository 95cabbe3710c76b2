"""The oracle's beam search (oracle/ti_oracle_beam.cpp: beam_search_decode restated,
inference_engine.cpp:1912-2069, with softmax / top-k / top-p filtering :1798-1910) pinned to the
REFERENCE on the CPU.

tests/golden/beam_plumbing.npz holds what the compiled reference's own generate_beam_search
returned on the plumbing model (deterministic: beam search draws nothing).  Driven by the
reference's forward pass there -- all seq_len x vocab logits of forward_pass read as one
distribution (:1961-1966), restated by or_plumbing_forward_rows -- the oracle must return the
same results in the same order: same tokens (the plumbing logits are full of exact ties, so
this also pins the std::sort / priority_queue orders), finished flags, and the per-token
log-prob bit for bit (log_prob / n_new in float, :862-865).  tests/test_gpu_beam.py then holds
the engine's beam search to this oracle over the oracle's own decode logits.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32
PROMPT = [1, 15, 25, 35]


def test_oracle_beam_search_pinned_to_reference(oracle, golden):
    d = golden("beam_plumbing")
    V, H, layers = 1000, 256, 4

    def forward(toks):
        return oracle.plumbing_forward_rows(V, H, layers, len(toks))

    for i in range(int(d["n"][0])):
        mn, beam, T, k, p, lpen = (float(x) for x in d[f"cfg{i}"])
        mn, beam, k = int(mn), int(beam), int(k)
        res, _ = oracle.beam_search(forward, PROMPT, mn, beam, T, k, p, lpen, eos=2)
        toks, fin, lps = d[f"tokens{i}"], d[f"finished{i}"], d[f"logprob{i}"]
        assert len(res) == len(toks), i
        for r, (rt, rlp, _rs, rf) in enumerate(res):
            want = [int(t) for t in toks[r] if t >= 0]
            assert rt == want, (i, r, rt, want)
            assert rf == bool(fin[r]), (i, r)
            per_tok = f32(rlp) / f32(len(rt))
            assert per_tok.view(np.uint32) == f32(lps[r]).view(np.uint32), (i, r, per_tok, lps[r])


def test_oracle_beam_search_zero_new_tokens(oracle):
    """max_new_tokens = 0: the loop never runs and the prompt comes back as the one finished
    candidate with no new tokens (:1937, :2052-2057)."""
    res, _ = oracle.beam_search(lambda t: np.zeros(8, f32), PROMPT, 0, 3)
    assert res == [([], 0.0, 0.0, True)]
