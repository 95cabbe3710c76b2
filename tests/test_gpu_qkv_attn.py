"""QKV projection + decode attention in one launch (ti_qkv_attn_partials).

One decode stream (TinyLlama-1.1B GQA head_dim 64, Llama-2-7B MHA head_dim 128): the launch computes q / k / v
with the fused GEMV's arithmetic (TI_X_F16_FOLDED input, TI_EPI_QKV_ROPE_KV epilogue), writes the
new K / V row, and attends q to the old keys in its splits and to the step's own key in the last
split (from the k / v tiles' exchange granules); the O projection merges the splits
(TI_X_ATTN_SPLITS).  Checked against the unfused launches on the same inputs:
  * k_p, v_p bit-identical (same items, same order, same reduction and epilogue arithmetic);
  * the O output within the split-merge bound of test_gpu_fold.py (the staged activation differs by
    the fp16 rounding of each split's normalised row);
  * an engine with it on vs off, step by step, within the decode tolerance (TOL, test_gpu_engine.py).
Reference: inference_engine.cpp:203-279 (layer forward), 291-368 (compute_attention).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from test_gpu_engine import TOL

pytestmark = pytest.mark.gpu

f16 = np.float16
f32 = np.float32


def dev(ti, a):
    return ti.DeviceBuffer.from_array(np.ascontiguousarray(a))


def gemm(ti, td, sd, bits, x_ptr, x_kind, ldx, M, N, K, ep, eps=1e-5):
    ti.check(ti.lib().ti_gemm_wq_a16(td.ptr, sd.ptr, bits, x_ptr, x_kind, ldx, None, eps, M, N, K, C.byref(ep), None))
    ti.sync()


@pytest.mark.parametrize("bits,K,heads,kv_heads,p,splits,hd", [
    (8, 2048, 32, 4, 2047, 8, 64),    # TinyLlama-1.1B at the bench position
    (8, 2048, 32, 4, 300, 8, 64),
    (4, 2048, 32, 4, 777, 8, 64),
    (8, 1024, 16, 4, 5, 4, 64),       # short: most splits empty
    (8, 2048, 32, 4, 0, 8, 64),       # first token: every split empty, O merges the new key alone
    (4, 4096, 32, 32, 2047, 8, 128),  # Llama-2-7B (MHA: every workgroup a k and a v tile)
    (4, 4096, 32, 32, 3, 8, 128),
    (8, 4096, 32, 32, 1000, 8, 128),
])
def test_fused_matches_unfused_launches(ti, oracle, bits, K, heads, kv_heads, p, splits, hd):
    rng = np.random.RandomState(bits * 1000 + p + heads + hd)
    max_seq, H, eps = 2048, 1024, 1e-5
    assert ti.lib().ti_qkv_attn_supported(bits, K, heads, kv_heads, hd, splits) == 1
    qd, kvd = heads * hd, kv_heads * hd
    N = qd + 2 * kvd
    w = (rng.standard_normal((K, N)) * 0.03).astype(f32)
    t, sc = ti.wpack_host(w, bits)
    td, sd = dev(ti, t), dev(ti, sc)
    fx = (rng.standard_normal(K) * 0.5).astype(f16)
    ss = np.abs(rng.standard_normal(3)).astype(f32) * (K / 3)
    fxd, ssd = dev(ti, fx), dev(ti, ss)
    cs = ti.rope_table(np.arange(max_seq), hd, 10000.0).reshape(max_seq, hd)
    csd = dev(ti, cs)
    pos = np.array([p], np.int32)
    pd = dev(ti, pos)
    kc = (rng.standard_normal((kv_heads, max_seq, hd)) * 0.5).astype(f16)
    vc = rng.standard_normal((kv_heads, max_seq, hd)).astype(f16)
    L_ = ti.lib()

    # unfused: QKV GEMV (q, cache row p), ti_attn_decode_partials over [0, p], O with TI_X_ATTN_SPLITS
    kua, vua = dev(ti, kc), dev(ti, vc)
    qb = ti.DeviceBuffer(qd * 4)
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_QKV_ROPE_KV, qd, qb.ptr
    ep.q_dim, ep.kv_dim, ep.head_dim, ep.max_seq = qd, kvd, hd, max_seq
    ep.pos, ep.rope_cs, ep.k_cache, ep.v_cache, ep.kv_stream_stride = pd.ptr, csd.ptr, kua.ptr, vua.ptr, 0
    ep.ss_in, ep.n_ss = ssd.ptr, ss.size
    gemm(ti, td, sd, bits, fxd.ptr, ti.X_F16_FOLDED, K, 1, N, K, ep, eps)
    po = ti.DeviceBuffer(heads * splits * hd * 2)
    pml = ti.DeviceBuffer(heads * splits * 8)
    ti.check(L_.ti_attn_decode_partials(qb.ptr, kua.ptr, vua.ptr, 0, max_seq, pd.ptr, 1, heads, kv_heads, hd, splits,
                                        po.ptr, pml.ptr, None))

    # fused
    kfu, vfu = dev(ti, kc), dev(ti, vc)
    po2 = ti.DeviceBuffer(L_.ti_qkv_attn_part_o_elems(heads, hd, splits) * 2)
    pml2 = ti.DeviceBuffer(L_.ti_qkv_attn_part_ml_elems(heads, hd, splits) * 4)
    xg = ti.DeviceBuffer(L_.ti_qkv_attn_xchg_bytes(heads, splits))
    xg.zero()
    ti.check(L_.ti_qkv_attn_partials(td.ptr, sd.ptr, bits, fxd.ptr, ssd.ptr, ss.size, eps, csd.ptr, pd.ptr, kfu.ptr,
                                     vfu.ptr, max_seq, K, heads, kv_heads, hd, splits, po2.ptr, pml2.ptr, xg.ptr, None))
    ti.sync()

    # k_p / v_p bit-identical, the rest of the caches untouched
    for a, b in ((kua, kfu), (vua, vfu)):
        assert np.array_equal(a.download(np.uint16, kc.shape), b.download(np.uint16, kc.shape))

    # O projection of both against the merged attention (ti_attn_decode over [0, p], fp16 out)
    wo = (rng.standard_normal((qd, H)) * 0.03).astype(f32)
    to, so = ti.wpack_host(wo, 4)
    tod, sod = dev(ti, to), dev(ti, so)
    ya, yb = ti.DeviceBuffer(H * 4), ti.DeviceBuffer(H * 4)
    ea = ti.Epilogue()
    ea.kind, ea.ldo, ea.out, ea.ss_in, ea.n_ss, ea.head_dim = ti.EPI_STORE_F32, H, ya.ptr, pml.ptr, splits, hd
    gemm(ti, tod, sod, 4, po.ptr, ti.X_ATTN_SPLITS, qd, 1, H, qd, ea)
    eb = ti.Epilogue()
    eb.kind, eb.ldo, eb.out, eb.ss_in, eb.n_ss, eb.head_dim = ti.EPI_STORE_F32, H, yb.ptr, pml2.ptr, splits, hd
    gemm(ti, tod, sod, 4, po2.ptr, ti.X_ATTN_SPLITS, qd, 1, H, qd, eb)
    ws = ti.DeviceBuffer(L_.ti_attn_workspace_bytes(1, heads, hd, splits))
    ws.zero()
    out = ti.DeviceBuffer(qd * 2)
    ti.check(L_.ti_attn_decode(qb.ptr, kua.ptr, vua.ptr, 0, max_seq, pd.ptr, 1, heads, kv_heads, hd, splits, ws.ptr,
                               out.ptr, None))
    ti.sync()
    xa = out.download(f16, qd).astype(np.float64)
    q4, s4 = oracle.quantize_groups(wo, 4)
    wf = np.abs(oracle.dequantize_groups(q4, s4).astype(np.float64))
    got, ref = yb.download(f32, H).astype(np.float64), ya.download(f32, H).astype(np.float64)
    assert np.all(np.isfinite(got))
    bound = 2.5e-3 * (np.abs(xa) @ wf) + 1e-6
    err = np.abs(got - ref)
    assert np.all(err <= bound), f"max err {err.max()} (bound {bound.min()})"


CFGS = {   # vocab, hidden, layers, heads, kv_heads, head_dim, inter, bits, max_seq
    "tl_shape_w8": (32000, 2048, 3, 32, 4, 64, 5632, 8, 256),
    "tl_shape_w4": (32000, 2048, 2, 32, 4, 64, 5632, 4, 256),
    "gqa16_w8": (4096, 1024, 2, 16, 4, 64, 2816, 8, 256),
    "l2_shape_w4": (32000, 4096, 2, 32, 32, 128, 11008, 4, 512),   # 8 splits from 512 positions
}


@pytest.mark.parametrize("name", list(CFGS))
def test_engine_qkv_attn_matches_unfused_steps(ti, name):
    """Twin engines (fused QKV + attention on / off) fed the same tokens: logits within the decode
    tolerance every step from position 0 (all old-key splits empty) on, greedy argmax equal wherever
    the top-2 margin exceeds twice it."""
    v, h, l, nh, nkv, hd, inter, bits, ms = CFGS[name]
    eng = {}
    for on in (True, False):
        e = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=bits, max_seq=ms, max_batch=1)
        e.synth(0x9a11, 0.1)
        e.set_prefill(0)
        assert e.set_qkv_attn(on) is on
        eng[on] = e
    toks = [3, 17, 99, 5]
    for pos in range(40):
        lf = eng[True].step([toks[pos]], [pos])[0].astype(np.float64)
        lu = eng[False].step([toks[pos]], [pos])[0].astype(np.float64)
        tol = TOL * float(np.max(np.abs(lu)))
        assert float(np.max(np.abs(lf - lu))) <= tol, pos
        srt = np.sort(lu)
        if srt[-1] - srt[-2] > 2 * tol:
            assert int(np.argmax(lf)) == int(np.argmax(lu)), pos
        if pos + 1 >= len(toks):
            toks.append(int(np.argmax(lu)))
    for e in eng.values():
        e.close()


def test_qkv_attn_off_paths(ti):
    """Not taken where it does not apply: splits that do not divide into the q tiles (head_dim 128 at
    4 splits), int16 weights, fold off."""
    e = ti.Engine(4096, 1024, 1, 8, 8, 128, 2816, bits=4, max_seq=256, max_batch=1)
    assert e.set_qkv_attn(True) is False
    e.close()
    e = ti.Engine(4096, 1024, 1, 16, 4, 64, 2816, bits=16, max_seq=256, max_batch=1)
    assert e.set_qkv_attn(True) is False
    e.close()
    e = ti.Engine(4096, 1024, 1, 16, 4, 64, 2816, bits=8, max_seq=256, max_batch=1)
    assert e.set_qkv_attn(True) is True
    e.set_fold(False)
    assert e.set_qkv_attn(None) is False
    e.close()


def test_qkv_attn_lost_sibling_is_reported_and_recovered(ti, monkeypatch):
    """Every wait in the launch is bounded: a workgroup that withholds its q part (TI_QA_DROP, test
    hook) leaves its siblings to time out -- the launch completes, the engine reports the step as failed
    (TI_ERR_HIP, the exchange's error word) and zeroes the exchange, and the step re-run and the next
    ones match a fresh engine's bit for bit."""
    v, h, l, nh, nkv, hd, inter, bits, ms = CFGS["gqa16_w8"]

    def make():
        e = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=bits, max_seq=ms, max_batch=1)
        e.synth(0x1057, 0.1)
        e.set_prefill(0)
        assert e.set_qkv_attn(True) is True
        return e

    bad, ref = make(), make()
    monkeypatch.setenv("TI_QA_DROP", "3")
    with pytest.raises(Exception, match="exchange timed out"):
        bad.step([7], [0])
    monkeypatch.delenv("TI_QA_DROP")
    bad.set_qkv_attn(False)   # (drops the step graph captured with the hook)
    assert bad.set_qkv_attn(True) is True
    # (the failed step wrote layers 1.. of position 0's K / V from a wrong head 0: the step is re-run)
    for pos, tok in ((0, 7), (1, 11), (2, 5)):
        a = bad.step([tok], [pos])[0]
        b = ref.step([tok], [pos])[0]
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), pos
    bad.close()
    ref.close()
