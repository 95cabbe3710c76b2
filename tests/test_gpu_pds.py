"""Persistent decode layers (ti_pds_decode, pds.hip) against the per-layer launches.

The persistent launch runs every decode layer of a single-stream step with the same arithmetic,
item for item, as the per-layer launches with the folded rms_norm and split-partials hand-offs,
so twin engines fed the same tokens must give bit-identical logits at every step (positions
crossing the 8 attention splits' boundaries, position 0 included), identical greedy tokens, and
no hand-off timeout.  The per-layer path itself is held to the oracle by test_gpu_engine.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CFGS = {
    # name: vocab, hidden, layers, heads, kv_heads, head_dim, inter, bits
    "small": (512, 256, 2, 2, 2, 128, 512, 4),                 # MHA head-group QKV mapping
    "l2_shape": (32000, 4096, 2, 32, 32, 128, 11008, 4),       # Llama-2-7B layer shape
    "tl_shape": (32000, 2048, 2, 32, 4, 64, 5632, 8),          # TinyLlama-1.1B: INT8, GQA 8, head_dim 64
    "gqa_w4_hd64": (512, 256, 2, 4, 2, 64, 768, 4),            # GQA 2, hd 64, fewer O tiles than CUs
    "gqa_w8_hd128": (1024, 512, 2, 4, 1, 128, 1024, 8),        # GQA 4, INT8, hd 128
}


def _twins(ti, name, max_seq):
    v, h, l, nh, nkv, hd, inter, bits = CFGS[name]
    eng = {}
    for on in (True, False):
        e = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=bits, max_seq=max_seq, max_batch=1, attn_splits=8)
        e.synth(0x7157, 0.1)
        e.set_prefill(0)
        assert e.set_fold(True)
        assert e.set_pds(on) is on
        eng[on] = e
    return eng


@pytest.mark.parametrize("name", list(CFGS))
def test_pds_steps_bit_identical(ti, name):
    eng = _twins(ti, name, 256)
    toks = [3, 17, 99, 5]
    for pos in range(40):
        a = eng[True].step([toks[pos]], [pos])[0]
        b = eng[False].step([toks[pos]], [pos])[0]
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), pos
        if pos + 1 >= len(toks):
            toks.append(int(np.argmax(b)))
    assert eng[True].pds_error() == 0
    ga = eng[True].generate([[1, 2, 3]], 12)
    gb = eng[False].generate([[1, 2, 3]], 12)
    assert np.array_equal(np.asarray(ga), np.asarray(gb))
    assert eng[True].pds_error() == 0
    for e in eng.values():
        e.close()


@pytest.mark.parametrize("name", ["l2_shape", "tl_shape"])
def test_pds_long_context_replay(ti, name):
    """7B layer shape over a 2048-slot synthetic KV cache (the bench's configuration, 2 layers):
    replayed steps at position 2047 give the same argmax token with the persistent launch on and
    off, and repeated launches (monotonic hand-off counters) never time out."""
    v, h, l, nh, nkv, hd, inter, bits = CFGS[name]
    toks = {}
    for on in (True, False):
        e = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=bits, max_seq=2048, max_batch=1)
        e.synth(0x7157, 0.1)
        assert e.set_pds(on) is on
        e.fill_kv(0, 2047, 0x5eed)
        e.replay_prepare(1, 2048, 7)
        e.replay_run(64)
        e.sync()
        toks[on] = e.last_tokens(1)
        if on:
            assert e.pds_error() == 0
        e.close()
    assert np.array_equal(toks[True], toks[False])


def test_pds_timeout_is_fatal(ti, monkeypatch):
    """A hand-off wait that timed out (error word forced, TI_PDS_FORCE_ERR) must not hand back
    tokens: generate / step raise, the engine turns persistent decode off and resets the
    hand-off state, and the next call runs on the per-layer graph with correct results."""
    v, h, l, nh, nkv, hd, inter, _bits = CFGS["l2_shape"]
    ref = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=4, max_seq=256, max_batch=1, attn_splits=8)
    ref.synth(0x7157, 0.1)
    want = np.asarray(ref.generate([[1, 2, 3]], 6))
    ref.close()
    e = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=4, max_seq=256, max_batch=1, attn_splits=8)
    e.synth(0x7157, 0.1)
    monkeypatch.setenv("TI_PDS_FORCE_ERR", "1")
    assert e.set_pds(True) is True
    monkeypatch.delenv("TI_PDS_FORCE_ERR")
    with pytest.raises(ti.TiError, match="persistent decode"):
        e.generate([[1, 2, 3]], 6)
    assert e.set_pds(None) is False          # turned off by the failure
    assert e.pds_error() == 0                # state reset
    assert np.array_equal(np.asarray(e.generate([[1, 2, 3]], 6)), want)
    monkeypatch.setenv("TI_PDS_FORCE_ERR", "1")
    assert e.set_pds(True) is True
    monkeypatch.delenv("TI_PDS_FORCE_ERR")
    with pytest.raises(ti.TiError, match="persistent decode"):
        e.step([5], [0])
    e.close()


def test_pds_lost_producer_costs_one_timeout(ti, monkeypatch):
    """A producer that never publishes mid-launch (TI_PDS_FORCE_ERR=2: workgroup 0 withholds its
    layer-0 down-projection granules): every other workgroup waits on them, the first expiry (~50 ms)
    marks the launch dead and every later wait of every workgroup passes at once.  The
    call fails with the fatal hand-off error within a few timeouts, not one per wait, and the engine
    falls back to the per-layer graph with correct results."""
    import time
    v, h, l, nh, nkv, hd, inter, _bits = CFGS["l2_shape"]
    ref = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=4, max_seq=256, max_batch=1, attn_splits=8)
    ref.synth(0x7157, 0.1)
    want = np.asarray(ref.generate([[1, 2, 3]], 4))
    ref.close()
    e = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=4, max_seq=256, max_batch=1, attn_splits=8)
    e.synth(0x7157, 0.1)
    monkeypatch.setenv("TI_PDS_FORCE_ERR", "2")
    assert e.set_pds(True) is True
    monkeypatch.delenv("TI_PDS_FORCE_ERR")
    t0 = time.perf_counter()
    with pytest.raises(ti.TiError, match="persistent decode"):
        e.step([5], [0])
    assert time.perf_counter() - t0 < 1.0
    assert e.set_pds(None) is False
    assert np.array_equal(np.asarray(e.generate([[1, 2, 3]], 4)), want)
    e.close()
