"""QKV projection + attention in one launch (ti_hip.h ti_qkv_attn_fused, ti_engine_set_qkv_attn).

The fused launch runs the same QKV GEMV body (folded input, RoPE + KV-append epilogue) and the
same attention split body (partials mode, splits = head_dim / 16) as the two launches it
replaces -- ti_gemm_wq_a16(TI_X_F16_FOLDED, TI_EPI_QKV_ROPE_KV) followed by
ti_attn_decode_partials -- with the head's workgroups handing q / K / V over through a counter
instead of a launch boundary.  Same inputs, same arithmetic in the same order: every output
(q, the appended K/V rows, the split rows and (max, sum) pairs) must be bit-identical, and the
hand-off counters must be left at zero for the next launch.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

f16 = np.float16
f32 = np.float32


def dev(ti, a):
    return ti.DeviceBuffer.from_array(np.ascontiguousarray(a))


@pytest.mark.parametrize("heads,hd,K,L", [(32, 128, 4096, 2048), (32, 128, 4096, 5), (4, 64, 256, 300),
                                          (8, 128, 1024, 777)])
def test_fused_matches_qkv_then_partials(ti, heads, hd, K, L):
    rng = np.random.RandomState(heads + hd + L)
    qd = heads * hd
    N, S, max_seq = 3 * qd, hd // 16, max(L, 64)
    w = (rng.standard_normal((K, N)) * 0.03).astype(f32)
    t, sc = ti.wpack_host(w, 4)
    td, sd = dev(ti, t), dev(ti, sc)
    x = rng.standard_normal(K).astype(f16)
    ss = (np.abs(rng.standard_normal(3)) * K / 3).astype(f32)
    xd, ssd = dev(ti, x), dev(ti, ss)
    cs = dev(ti, ti.rope_table(np.arange(max_seq, dtype=f32), hd, 10000.0))
    pos = dev(ti, np.array([L - 1], np.int32))
    kc0 = (rng.standard_normal((heads, max_seq, hd)) * 0.5).astype(f16)
    vc0 = rng.standard_normal((heads, max_seq, hd)).astype(f16)
    out = {}
    L_ = ti.lib()
    ctr = ti.DeviceBuffer(heads * 16 * 4)
    ctr.zero()
    abort = ti.DeviceBuffer(4)
    abort.zero()
    for fused in (True, False):
        q, kc, vc = ti.DeviceBuffer(qd * 4), dev(ti, kc0), dev(ti, vc0)
        po, pml = ti.DeviceBuffer(heads * S * hd * 2), ti.DeviceBuffer(heads * S * 8)
        ep = ti.Epilogue()
        ep.kind, ep.ldo, ep.out = ti.EPI_QKV_ROPE_KV, qd, q.ptr
        ep.q_dim, ep.kv_dim, ep.head_dim, ep.max_seq = qd, qd, hd, max_seq
        ep.pos, ep.rope_cs, ep.k_cache, ep.v_cache, ep.kv_stream_stride = pos.ptr, cs.ptr, kc.ptr, vc.ptr, qd * max_seq
        ep.ss_in, ep.n_ss = ssd.ptr, ss.size
        if fused:
            for _ in range(2):   # the second launch finds the counters re-armed
                ti.check(L_.ti_qkv_attn_fused(td.ptr, sd.ptr, xd.ptr, 1e-5, K, C.byref(ep), po.ptr, pml.ptr, ctr.ptr,
                                              abort.ptr, None))
        else:
            ti.check(L_.ti_gemm_wq_a16(td.ptr, sd.ptr, 4, xd.ptr, ti.X_F16_FOLDED, K, None, 1e-5, 1, N, K, C.byref(ep),
                                       None))
            ti.check(L_.ti_attn_decode_partials(q.ptr, kc.ptr, vc.ptr, qd * max_seq, max_seq, pos.ptr, 1, heads, heads,
                                                hd, S, po.ptr, pml.ptr, None))
        ti.sync()
        out[fused] = (q.download(f32, qd), kc.download(f16, kc0.shape)[:, L - 1], vc.download(f16, vc0.shape)[:, L - 1],
                      po.download(f16, (heads, S, hd)), pml.download(f32, (heads, S, 2)))
    assert abort.download(np.uint32, 1)[0] == 0
    assert np.all(ctr.download(np.uint32, heads * 16) == 0)
    for name, a, b in zip(("q", "k", "v", "part_o", "part_ml"), out[True], out[False]):
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), name
    # the rows really are this step's: K/V at pos differ from the seeded cache
    assert not np.array_equal(out[True][1], kc0[:, L - 1])


def test_fused_rejects_unsupported_shapes(ti):
    L_ = ti.lib()
    ep = ti.Epilogue()
    ep.kind = ti.EPI_QKV_ROPE_KV
    buf = ti.DeviceBuffer(1 << 16)
    ep.out = ep.pos = ep.rope_cs = ep.k_cache = ep.v_cache = ep.ss_in = buf.ptr
    ep.q_dim, ep.kv_dim, ep.head_dim, ep.max_seq, ep.ldo, ep.n_ss = 256, 128, 64, 16, 256, 1   # GQA: kv != q
    ep.kv_stream_stride = 256 * 16
    rc = L_.ti_qkv_attn_fused(buf.ptr, buf.ptr, buf.ptr, 1e-5, 256, C.byref(ep), buf.ptr, buf.ptr, buf.ptr, buf.ptr,
                              None)
    assert rc != 0 and b"kv_dim" in L_.ti_last_error()
    ep.kv_dim, ep.n_ss = 256, 0                                                                # no ss partials
    rc = L_.ti_qkv_attn_fused(buf.ptr, buf.ptr, buf.ptr, 1e-5, 256, C.byref(ep), buf.ptr, buf.ptr, buf.ptr, buf.ptr,
                              None)
    assert rc != 0


CFGS = {
    # name: vocab, hidden, layers, heads, kv_heads, head_dim, inter
    "mha_hd64": (512, 256, 2, 4, 4, 64, 512),
    "l2_shape": (32000, 4096, 2, 32, 32, 128, 11008),
}


@pytest.mark.parametrize("name", list(CFGS))
def test_engine_fused_steps_bit_identical(ti, name):
    """Twin engines (attention splits = head_dim / 16 in both), fused on vs off, fed the same
    tokens: logits bit-identical at every step; then greedy generate() agrees token for token."""
    v, h, l, nh, nkv, hd, inter = CFGS[name]
    eng = {}
    for on in (True, False):
        e = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=4, max_seq=256, max_batch=1, attn_splits=hd // 16)
        e.synth(0x7157, 0.1)
        e.set_prefill(0)
        assert e.set_fold(True)
        assert e.set_qkv_attn(on) is on
        eng[on] = e
    toks = [3, 17, 99, 5]
    for pos in range(24):
        a = eng[True].step([toks[pos]], [pos])[0]
        b = eng[False].step([toks[pos]], [pos])[0]
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), pos
        if pos + 1 >= len(toks):
            toks.append(int(np.argmax(b)))
    ga = eng[True].generate([[1, 2, 3]], 12)
    gb = eng[False].generate([[1, 2, 3]], 12)
    assert np.array_equal(np.asarray(ga), np.asarray(gb))
    for e in eng.values():
        e.close()
