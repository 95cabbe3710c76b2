"""Beam search (ti_engine_beam_search, C++ InferenceEngine::generate_beam_search) against a
restatement of the reference's beam_search_decode (inference_engine.cpp:1912-2069) and its
softmax / apply_top_k_filtering / apply_top_p_filtering helpers (:1798-1910), driven by the
same engine's forward passes (the last position's logits of each candidate, computed by
generate(candidate, 1)).

The restatement is float32 numpy in the reference's operation order (sequential sums via
cumsum); numpy's exp may differ from glibc's by an ulp, so beams must match exactly and
log-probabilities / scores to 1e-5 relative.  (The reference itself reads seq_len x vocab
logits of its full-sequence forward pass as one distribution, a bug not reproduced; its
llama forward pass is broken anyway)
"""
from __future__ import annotations

import heapq
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

f32 = np.float32


def _softmax(lg):
    mx = lg.max()
    p = np.exp((lg - mx).astype(f32)).astype(f32)
    s = np.cumsum(p, dtype=f32)[-1]
    return (p / s).astype(f32) if s > 0 else p


def _renorm(f):
    s = np.cumsum(f, dtype=f32)[-1]
    return (f / s).astype(f32) if s > 0 else f


def _order(p):            # std::sort descending by probability (ties: lower index first here)
    return sorted(range(len(p)), key=lambda i: (-float(p[i]), i))


def _top_k(p, k):
    if k >= len(p):
        return p
    f = p.copy()
    for i in _order(p)[k:]:
        f[i] = 0
    return _renorm(f)


def _top_p(p, top_p):
    if top_p >= 1.0:
        return p
    cum, keep = f32(0), np.zeros(len(p), bool)
    for i in _order(p):
        cum = f32(cum + p[i])
        keep[i] = True
        if cum >= f32(top_p):
            break
    f = np.where(keep, p, f32(0)).astype(f32)
    return _renorm(f)


def ref_beam_search(forward, prompt, max_new, beam_size, T, top_k, top_p, lp_pow, eos):
    heap, tie = [], 0
    heapq.heappush(heap, (-0.0, tie, list(prompt), f32(0), f32(0), False))
    done = []
    for _ in range(max_new):
        cur = []
        while heap:
            cur.append(heapq.heappop(heap))
        if not cur:
            break
        nxt = []
        for (_, _, toks, lpb, _, fin) in cur:
            if fin:
                done.append((toks, lpb, f32(0), fin))
                continue
            lg = forward(toks).astype(f32)
            if T != 1.0:
                lg = (lg / f32(T)).astype(f32)
            p = _softmax(lg)
            if 0 < top_k < len(p):
                p = _top_k(p, top_k)
            if top_p < 1.0:
                p = _top_p(p, top_p)
            cands = [i for i in _order(p) if p[i] > 0][:beam_size]
            for i in cands:
                nt = toks + [i]
                nl = f32(lpb + f32(math.log(float(p[i]))))
                nxt.append([nt, nl, f32(0), i == eos or len(nt) >= len(prompt) + max_new])
        for c in nxt:
            c[2] = f32(c[1] / f32(len(c[0]) ** lp_pow))
        nxt.sort(key=lambda c: -float(c[2]))
        for c in nxt[:beam_size]:
            if c[3]:
                done.append(tuple(c))
            else:
                tie += 1
                heapq.heappush(heap, (-float(c[1]), tie, c[0], c[1], c[2], False))
        if len(done) >= beam_size:
            break
    while heap:
        _, _, toks, lpb, sc, _ = heapq.heappop(heap)
        done.append((toks, lpb, sc, True))
    done.sort(key=lambda c: -float(c[2]))
    return [(c[0][len(prompt):], float(c[1]), float(c[2]), bool(c[3])) for c in done[:beam_size]]


@pytest.mark.parametrize("beam,T,k,p,lp", [(3, 1.0, 0, 1.0, 1.0), (4, 0.8, 50, 0.95, 0.6), (2, 1.2, 8, 1.0, 1.5)])
def test_beam_search_matches_reference_logic(ti, beam, T, k, p, lp):
    e = ti.Engine(512, 256, 2, 4, 2, 64, 512, bits=4, max_seq=64, max_batch=1)
    e.synth(0x7157, 0.1)
    prompt, new = [3, 17, 99, 5], 6

    def forward(toks):
        return e.generate([toks], 1, want_logits=True)[1][0]

    want = ref_beam_search(forward, prompt, new, beam, T, k, p, lp, 2)
    got = e.beam_search(prompt, new, beam, T, k, p, lp, 2)
    e.close()
    assert len(got) == len(want)
    for (gt, gl, gs, gf), (wt, wl, ws, wf) in zip(got, want):
        assert gt == wt and gf == wf
        assert abs(gl - wl) <= 1e-5 * max(1.0, abs(wl)) and abs(gs - ws) <= 1e-5 * max(1.0, abs(ws))
