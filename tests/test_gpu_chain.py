"""Chained decode steps (ti_hip.h ti_chain, ti_engine_set_chain) against the hipGraph path.

A chained step issues its launches with hipExtAnyOrderLaunch and orders them in-kernel
(counter waits, write-through hand-offs).  The arithmetic is the graph path's, so tokens and
logits must be BIT-identical between the two; any stale read of a handed-off byte (the
residual, q, the freshly appended K/V row, the argmax keys, the step counter) shows up as a
difference.  Replay mode rewrites the same KV position every step with new values: the
strongest staleness check.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CFGS = {
    # name: vocab, hidden, layers, heads, kv_heads, head_dim, inter, bits
    "mini_gqa_w4": (512, 256, 2, 4, 2, 64, 512, 4),
    "tl_shape_w8": (32000, 2048, 3, 32, 4, 64, 5632, 8),
    "l2_shape_w4": (32000, 4096, 2, 32, 32, 128, 11008, 4),
    "l3_shape_w4": (128256, 4096, 2, 32, 8, 128, 14336, 4),
}


def make(ti, name, max_seq=640):
    v, h, l, nh, nkv, hd, inter, bits = CFGS[name]
    e = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=bits, max_seq=max_seq, max_batch=1)
    e.synth(0x7157, 0.1)
    e.set_fold(False)   # chained launches run the unfolded kernels (ti_engine_set_fold)
    return e


@pytest.mark.parametrize("name", list(CFGS))
def test_chain_active_for_single_stream(ti, name):
    e = make(ti, name, max_seq=64)
    assert e.set_chain() is False          # default: the replayed graph
    assert e.set_chain(True) is True
    assert e.set_chain() is True
    assert e.set_chain(False) is False
    assert e.set_chain(True) is True
    e.close()


@pytest.mark.parametrize("name", list(CFGS))
def test_chained_generate_is_bit_identical_to_graph(ti, name):
    prompt = [[3, 17, 99, 5, 250]]
    e = make(ti, name)
    e.set_chain(False)
    e.set_prefill(0)
    ref_tok, ref_lg = e.generate(prompt, 40, want_logits=True)
    e.set_chain(True)
    got_tok, got_lg = e.generate(prompt, 40, want_logits=True)
    e.close()
    assert got_tok.tolist() == ref_tok.tolist()
    assert np.array_equal(got_lg, ref_lg)


@pytest.mark.parametrize("name", ["tl_shape_w8", "l2_shape_w4"])
def test_chained_replay_rewrites_kv_slot_without_stale_reads(ti, name):
    res = {}
    for chain in (False, True):
        e = make(ti, name)
        e.fill_kv(0, 600, 1234)
        e.set_chain(chain)
        e.replay_prepare(1, 600, 7)
        e.replay_run(48)
        e.sync()
        tok = e.last_tokens(1)
        lg = e.step([int(tok[0])], [599])   # one more (unchained first-step) decode at the same slot
        res[chain] = (tok.tolist(), lg)
        e.close()
    assert res[True][0] == res[False][0]
    assert np.array_equal(res[True][1], res[False][1])


def test_chained_steps_interleave_with_graph_steps(ti):
    """Chained runs and graph runs on one engine hand state over through the stream order."""
    e = make(ti, "tl_shape_w8")
    e.set_prefill(0)
    e.set_chain(False)
    ref = e.generate([[1, 2, 3]], 24)
    outs = []
    for chain in (True, False, True):
        e.set_chain(chain)
        t = e.generate([[1, 2, 3]], 24)
        outs.append(t.tolist())
    e.close()
    assert all(o == ref.tolist() for o in outs)
