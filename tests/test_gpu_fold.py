"""Folded rms_norm hand-off (ti_hip.h TI_X_F16_FOLDED, ti_engine_set_fold).

The producer epilogue (TI_EPI_RESID_F32 with fold_x) writes the residual h, fp16(h * nw) and
its workgroups' partial sums of h^2; the consumer stages those fp16 rows and divides its
outputs by sqrt(sum / K + eps).  Mathematically this is the fused TI_X_F32_RMSNORM prologue
(rms_norm, tensor_engine.cpp:1452-1508, then matmul) with the division moved behind the GEMM,
so the two agree up to the fp16 rounding of the staged activation: one fp16 ulp per element,
the bound of test_gpu_kernels.py's rms_norm prologue test.  The fold outputs themselves are
checked exactly (fp16 products) and to fp32 summation order (sum of squares).
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


def gemm(ti, td, sd, bits, x_ptr, x_kind, ldx, M, N, K, ep, norm_ptr=None, eps=1e-5):
    ti.check(ti.lib().ti_gemm_wq_a16(td.ptr, sd.ptr, bits, x_ptr, x_kind, ldx, norm_ptr, eps, M, N, K,
                                     C.byref(ep), None))
    ti.sync()


@pytest.mark.parametrize("bits,H,Kp,N2", [(4, 4096, 4096, 12288), (4, 2048, 5632, 32000), (8, 4096, 11008, 2048)])
def test_fold_producer_and_consumer(ti, oracle, bits, H, Kp, N2):
    rng = np.random.RandomState(H + Kp + bits)
    # producer: h_new = r + W1 . a (the O / down projection), fold into fp16(h_new * nw)
    w1 = (rng.standard_normal((Kp, H)) * 0.03).astype(f32)
    a = rng.standard_normal((1, Kp)).astype(f16)
    r = (rng.standard_normal((1, H)) * 2).astype(f32)
    nw = (1 + 0.1 * rng.standard_normal(H)).astype(f32)
    t1, s1 = ti.wpack_host(w1, bits)
    hd, fxd, ssd = dev(ti, r), ti.DeviceBuffer(H * 2), ti.DeviceBuffer(256 * 4)
    ssd.zero()
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_RESID_F32, H, hd.ptr
    nwd, ad = dev(ti, nw), dev(ti, a)   # kept alive across the launches
    ep.fold_w, ep.fold_x, ep.fold_ss = nwd.ptr, fxd.ptr, ssd.ptr
    gemm(ti, dev(ti, t1), dev(ti, s1), bits, ad.ptr, ti.X_F16, Kp, 1, H, Kp, ep)
    h = hd.download(f32, (1, H))
    grid = ti.lib().ti_gemm_grid(1, H, Kp)
    assert 1 <= grid <= 256
    fx = fxd.download(f16, (1, H))
    # fp16 of the fp32 product; the hardware conversion may round an fp16-subnormal result
    # to the other neighbour (common.hpp f2h_soft): one fp16 ulp
    want = (h * nw).astype(f16)
    ulp = np.abs(fx.view(np.uint16).astype(np.int32) - want.view(np.uint16).astype(np.int32))
    assert ulp.max() <= 1 and np.count_nonzero(ulp) <= 4, np.flatnonzero(ulp)
    ss = ssd.download(f32, 256)
    np.testing.assert_allclose(ss[:grid].astype(np.float64).sum(), np.sum(h.astype(np.float64) ** 2), rtol=1e-5)
    assert np.all(ss[grid:] == 0)

    # consumer: y = W2 . rms_norm(h) via the fold, against the fused rms_norm prologue
    w2 = (rng.standard_normal((H, N2)) * 0.03).astype(f32)
    t2, s2 = ti.wpack_host(w2, bits)
    td2, sd2 = dev(ti, t2), dev(ti, s2)
    yf, yn = ti.DeviceBuffer(N2 * 4), ti.DeviceBuffer(N2 * 4)
    ec = ti.Epilogue()
    ec.kind, ec.ldo, ec.out, ec.ss_in, ec.n_ss = ti.EPI_STORE_F32, N2, yf.ptr, ssd.ptr, grid
    gemm(ti, td2, sd2, bits, fxd.ptr, ti.X_F16_FOLDED, H, 1, N2, H, ec)
    en = ti.Epilogue()
    en.kind, en.ldo, en.out = ti.EPI_STORE_F32, N2, yn.ptr
    gemm(ti, td2, sd2, bits, hd.ptr, ti.X_F32_RMSNORM, H, 1, N2, H, en, norm_ptr=nwd.ptr)
    got, ref = yf.download(f32, N2).astype(np.float64), yn.download(f32, N2).astype(np.float64)
    xa = oracle.rms_norm(h, nw).astype(f16).astype(np.float64)[0]
    q, sc = oracle.quantize_groups(w2, bits)
    wf = np.abs(oracle.dequantize_groups(q, sc).astype(np.float64))
    bound = 2.5e-3 * (np.abs(xa) @ wf) + 1e-6
    err = np.abs(got - ref)
    assert np.all(err <= bound), f"max err {err.max()} (bound {bound.min()})"


CFGS = {
    # name: vocab, hidden, layers, heads, kv_heads, head_dim, inter, bits
    "mini_gqa_w4": (512, 256, 2, 4, 2, 64, 512, 4),
    "tl_shape_w8": (32000, 2048, 3, 32, 4, 64, 5632, 8),
    "l2_shape_w4": (32000, 4096, 2, 32, 32, 128, 11008, 4),
}


@pytest.mark.parametrize("name", list(CFGS))
def test_engine_fold_matches_unfolded_steps(ti, name):
    """Fold on vs off on twin engines fed the same tokens step by step: logits within the
    decode tolerance (TOL of max |logit|, test_gpu_engine.py) every step, greedy argmax equal
    wherever the top-2 margin exceeds twice it (which the bound implies); then greedy generate() from the same prompt agrees on those steps."""
    v, h, l, nh, nkv, hd, inter, bits = CFGS[name]
    eng = {}
    for fold in (True, False):
        e = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=bits, max_seq=256, max_batch=1)
        e.synth(0x7157, 0.1)
        e.set_prefill(0)
        assert e.set_fold(fold) is fold
        eng[fold] = e
    toks = [3, 17, 99, 5]
    for pos in range(20):
        lf = eng[True].step([toks[pos]], [pos])[0].astype(np.float64)
        lu = eng[False].step([toks[pos]], [pos])[0].astype(np.float64)
        tol = TOL * float(np.max(np.abs(lu)))
        assert float(np.max(np.abs(lf - lu))) <= tol, pos
        srt = np.sort(lu)
        if srt[-1] - srt[-2] > 2 * tol:      # then the bound above decides the argmax
            assert int(np.argmax(lf)) == int(np.argmax(lu)), pos
        if pos + 1 >= len(toks):
            toks.append(int(np.argmax(lu)))
    for e in eng.values():
        e.close()


@pytest.mark.parametrize("heads,kv_heads,hd,L,splits", [(32, 32, 128, 2048, 8), (32, 32, 128, 5, 8),
                                                         (16, 4, 64, 300, 4), (32, 8, 128, 777, 3)])
def test_attention_partials_merged_by_o_projection(ti, oracle, heads, kv_heads, hd, L, splits):
    """ti_attn_decode_partials + the O projection with TI_X_ATTN_SPLITS against ti_attn_decode
    (merged in its own launch, fp16 out) + the O projection with TI_X_F16 on the same cache.
    The staged activation differs by the fp16 rounding of each split's normalised row (one
    fp16 ulp of the merged value) -- the rms_norm-prologue bound; L = 5 leaves splits empty."""
    rng = np.random.RandomState(heads + L + splits)
    max_seq, H = max(L, 64), 512
    q = rng.standard_normal((1, heads * hd)).astype(f32)
    kc = (rng.standard_normal((kv_heads, max_seq, hd)) * 0.5).astype(f16)
    vc = rng.standard_normal((kv_heads, max_seq, hd)).astype(f16)
    pos = np.array([L - 1], np.int32)
    qd, kd, vd, pd = dev(ti, q), dev(ti, kc), dev(ti, vc), dev(ti, pos)
    L_ = ti.lib()
    po = ti.DeviceBuffer(heads * splits * hd * 2)
    pml = ti.DeviceBuffer(heads * splits * 8)
    ti.check(L_.ti_attn_decode_partials(qd.ptr, kd.ptr, vd.ptr, 0, max_seq, pd.ptr, 1, heads, kv_heads, hd, splits,
                                        po.ptr, pml.ptr, None))
    ws = ti.DeviceBuffer(L_.ti_attn_workspace_bytes(1, heads, hd, splits))
    ws.zero()
    out = ti.DeviceBuffer(heads * hd * 2)
    ti.check(L_.ti_attn_decode(qd.ptr, kd.ptr, vd.ptr, 0, max_seq, pd.ptr, 1, heads, kv_heads, hd, splits, ws.ptr,
                               out.ptr, None))
    ti.sync()
    ml = pml.download(f32, (heads, splits, 2))
    chunk = -(-L // splits)
    for s in range(splits):
        if s * chunk >= L:   # empty split: (-inf, 0) and a zero row
            assert np.all(np.isneginf(ml[:, s, 0])) and np.all(ml[:, s, 1] == 0)
    K = heads * hd
    w = (rng.standard_normal((K, H)) * 0.03).astype(f32)
    t, sc = ti.wpack_host(w, 4)
    td, sd = dev(ti, t), dev(ti, sc)
    ya, yb = ti.DeviceBuffer(H * 4), ti.DeviceBuffer(H * 4)
    ea = ti.Epilogue()
    ea.kind, ea.ldo, ea.out, ea.ss_in, ea.n_ss, ea.head_dim = ti.EPI_STORE_F32, H, ya.ptr, pml.ptr, splits, hd
    gemm(ti, td, sd, 4, po.ptr, ti.X_ATTN_SPLITS, K, 1, H, K, ea)
    eb = ti.Epilogue()
    eb.kind, eb.ldo, eb.out = ti.EPI_STORE_F32, H, yb.ptr
    gemm(ti, td, sd, 4, out.ptr, ti.X_F16, K, 1, H, K, eb)
    xa = out.download(f16, K).astype(np.float64)
    q4, s4 = oracle.quantize_groups(w, 4)
    wf = np.abs(oracle.dequantize_groups(q4, s4).astype(np.float64))
    got, ref = ya.download(f32, H).astype(np.float64), yb.download(f32, H).astype(np.float64)
    bound = 2.5e-3 * (np.abs(xa) @ wf) + 1e-6
    err = np.abs(got - ref)
    assert np.all(err <= bound), f"max err {err.max()} (bound {bound.min()})"
