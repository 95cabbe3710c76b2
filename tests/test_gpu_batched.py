"""The batched-rows GEMM (gemv_mb_kernel: int4 x fp16 rows beyond the fused kernel's LDS
image, generate_batch's M = B decode, inference_engine.cpp:804-828) and its rms_norm prep,
through the ti_hip.h C-ABI, against the oracle's dequantized weights.

Tolerance as in test_gpu_kernels.py: the expected values use the same fp16 activations and
the oracle's exact int4 x scale weights in float64, so what is left is fp32 summation order
(|err| <= 2e-5 * sum_k |x_k w_k| + 1e-6); fp16 outputs rtol 2e-3."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from test_gpu_kernels import assert_close_dot, deq, dev

pytestmark = pytest.mark.gpu
f16, f32 = np.float16, np.float32


SPLITK_BYTES = 64 << 20
TICKET_BYTES = 256 * 1024   # TI_SPLITK_TICKET_BYTES


@pytest.fixture(scope="module")
def splitk_ws(ti):
    b = ti.DeviceBuffer(SPLITK_BYTES)
    b.zero()
    return b


def tile_plan(ti, M, N, K, ws_bytes=SPLITK_BYTES, bits=4):
    a, b, c = C.c_int(), C.c_int(), C.c_int()
    rc = ti.lib().ti_gemm_tile_plan(bits, M, N, K, ws_bytes, C.byref(a), C.byref(b), C.byref(c))
    return (a.value, b.value, c.value) if rc == 0 else None


def run(ti, tiles, scales, x16, M, N, K, ep, ws=None):
    """One call; with ws (the split-K workspace) its tickets must be left re-armed (zero)."""
    L = ti.lib()
    if ws is not None:
        ep.splitk_ws, ep.splitk_bytes = ws.ptr, ws.nbytes
    ti.check(L.ti_gemm_wq_a16(tiles.ptr, scales.ptr, 4, x16.ptr, ti.X_F16, K, None, 1e-5, M, N, K, C.byref(ep), None))
    ti.sync()
    if ws is not None:
        assert not ws.download(np.int32, (TICKET_BYTES // 4,)).any(), "split-K tickets not re-armed"


# (M, K, N): rows 17-32 (two 16-row blocks), long K at few rows (one block), ragged tiles per
# workgroup (N/16 not a multiple of the grid), a last k-chunk of fewer than 8 k-tiles,
# more tiles than 5 per workgroup (grid grows)
@pytest.mark.parametrize("M,K,N", [(17, 1024, 64), (32, 4096, 4096 + 48), (24, 1152, 4000), (8, 11008, 256),
                                   (3, 14336, 96), (20, 4096, 25600), (32, 384, 16), (64, 4096, 12288),
                                   (48, 11008, 4096 + 16), (33, 1152, 4000), (64, 384, 16), (64, 14336, 256),
                                   (40, 4096, 32000), (128, 4096, 4096), (200, 1152, 4000 + 16), (256, 11008, 512),
                                   (129, 384, 16),
                                   # tile kernel at prefill chunks: 128 / 64 columns per workgroup, ragged tiles and rows
                                   (512, 4096, 22016), (700, 4096, 12288 + 48), (1000, 1152, 4000 + 16),
                                   (1024, 384, 16),
                                   # split K (with the workspace): narrow outputs at 65-128 rows, ragged slices
                                   (65, 4096, 4096), (128, 11008, 4096 + 16), (100, 14336, 512), (96, 3200, 1040)])
@pytest.mark.parametrize("splitk", [False, True])
def test_batched_store(ti, oracle, splitk_ws, M, K, N, splitk):
    """Without a workspace: the batched-rows kernels (<= 64 rows) and the tile kernel; with one
    (the engine's form), the tile kernel splits K over workgroups where the plan
    (ti_gemm_tile_plan) says so."""
    rng = np.random.RandomState(M * 7 + K + N)
    w = (rng.standard_normal((K, N)) * 0.03).astype(f32)
    x = rng.standard_normal((M, K)).astype(f16)
    assert ti.lib().ti_gemm_max_rows(4, ti.X_F16, N, K) >= M
    tiles, scales = ti.wpack_host(w, 4)
    yd = ti.DeviceBuffer(M * N * 4)
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_STORE_F32, N, yd.ptr
    run(ti, dev(ti, tiles), dev(ti, scales), dev(ti, x), M, N, K, ep, splitk_ws if splitk else None)
    wf = deq(oracle, w, 4)
    xa = x.astype(f32)
    assert_close_dot(yd.download(f32, (M, N)), xa.astype(np.float64) @ wf.astype(np.float64), xa, wf)


def test_splitk_plans_split_narrow_outputs(ti):
    """Tile-kernel calls whose one-slice grid would leave most CUs idle (narrow outputs at 65-128
    rows) split K, within the workspace; wide or tall calls and 17..64 rows do not."""
    for M, N, K in [(65, 4096, 4096), (128, 4096, 4096), (128, 4096, 11008), (100, 512, 14336)]:
        wmr, tpw, ks = tile_plan(ti, M, N, K)
        assert ks > 1, (M, N, K)
        n_cb = -(-(N // 16) // ((8 // wmr) * tpw))
        n_rb = -(-M // (64 * wmr))
        assert ks * n_cb * n_rb * 8 * tpw * 4 * 64 * 16 + TICKET_BYTES <= SPLITK_BYTES
        assert tile_plan(ti, M, N, K, ws_bytes=0)[2] == 1            # no workspace: no split
    assert tile_plan(ti, 512, 22016, 4096)[2] == 1
    assert tile_plan(ti, 64, 4096, 4096) is None                      # batched-rows kernel
    assert ti.lib().ti_gemm_packed_rows(4, 64) == 1


@pytest.mark.parametrize("M,K,N", [(512, 1024, 12288), (256, 1152, 22016), (1000, 1024, 12288)])
def test_tile_three_tiles_per_wave(ti, oracle, M, K, N):
    """Shapes the planner gives 192-column workgroups (3 weight tiles per wave: the 7B QKV's 768
    tiles at 64 rows as exactly 256 workgroups; gate/up at 256 rows), ragged rows included."""
    plan = tile_plan(ti, M, N, K)
    assert plan is not None and plan[1] == 3, plan
    rng = np.random.RandomState(M + N)
    w = (rng.standard_normal((K, N)) * 0.03).astype(f32)
    x = rng.standard_normal((M, K)).astype(f16)
    tiles, scales = ti.wpack_host(w, 4)
    yd = ti.DeviceBuffer(M * N * 4)
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_STORE_F32, N, yd.ptr
    run(ti, dev(ti, tiles), dev(ti, scales), dev(ti, x), M, N, K, ep)
    wf = deq(oracle, w, 4)
    xa = x.astype(f32)
    assert_close_dot(yd.download(f32, (M, N)), xa.astype(np.float64) @ wf.astype(np.float64), xa, wf)


@pytest.mark.parametrize("M,K,N", [(32, 4096, 32000), (17, 1152, 50016), (25, 384, 34000)])
def test_tile_32_row_waves(ti, oracle, M, K, N):
    """Wide outputs at <= 32 rows take the tile kernel with 32-row waves (half the activation
    block per group); ragged rows and tiles."""
    L = ti.lib()   # the wide-output tile path (TI_GEMM_TILE_WIDE_MN), not the batched-rows kernel
    assert L.ti_gemm_packed_rows(4, M) == 1 and L.ti_gemm_packed_rows_for(4, M, N, K) == 0
    rng = np.random.RandomState(M + K)
    w = (rng.standard_normal((K, N)) * 0.03).astype(f32)
    x = rng.standard_normal((M, K)).astype(f16)
    tiles, scales = ti.wpack_host(w, 4)
    yd = ti.DeviceBuffer(M * N * 4)
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_STORE_F32, N, yd.ptr
    run(ti, dev(ti, tiles), dev(ti, scales), dev(ti, x), M, N, K, ep)
    wf = deq(oracle, w, 4)
    xa = x.astype(f32)
    assert_close_dot(yd.download(f32, (M, N)), xa.astype(np.float64) @ wf.astype(np.float64), xa, wf)


def test_tile_32_row_waves_epilogues(ti, oracle):
    """Residual add, SiLU * up (LDS-staged epilogues) and logits + argmax (per element) on the
    32-row-wave tile kernel."""
    M, K, N = 29, 2048, 30016
    assert ti.lib().ti_gemm_packed_rows_for(4, M, N, K) == 0   # (the SiLU call has 2 I = N outputs too)
    rng = np.random.RandomState(29)
    x = rng.standard_normal((M, K)).astype(f16)
    xd, xa = dev(ti, x), x.astype(np.float64)
    w = (rng.standard_normal((K, N)) * 0.03).astype(f32)
    tiles, scales = ti.wpack_host(w, 4)
    r = rng.standard_normal((M, N)).astype(f32)
    rd = dev(ti, r)
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_RESID_F32, N, rd.ptr
    run(ti, dev(ti, tiles), dev(ti, scales), xd, M, N, K, ep)
    wf = deq(oracle, w, 4)
    assert_close_dot(rd.download(f32, (M, N)) - r, xa @ wf.astype(np.float64), x.astype(f32), wf, rel=5e-5)
    I = N // 2
    g = (rng.standard_normal((K, I)) * 0.05).astype(f32)
    u = (rng.standard_normal((K, I)) * 0.05).astype(f32)
    tiles, scales = ti.wpack_host(g, 4, n_total=2 * I, row_map=ti.ROWS_INTERLEAVE8, row_offset=0)
    ti.wpack_host(u, 4, n_total=2 * I, row_map=ti.ROWS_INTERLEAVE8, row_offset=8, tiles=tiles, scales=scales)
    yd = ti.DeviceBuffer(M * I * 2)
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_SILU_MUL_F16, I, yd.ptr
    run(ti, dev(ti, tiles), dev(ti, scales), xd, M, 2 * I, K, ep)
    gg, uu = xa @ deq(oracle, g, 4).astype(np.float64), xa @ deq(oracle, u, 4).astype(np.float64)
    np.testing.assert_allclose(yd.download(f16, (M, I)).astype(np.float64), uu * (gg / (1 + np.exp(-gg))),
                               rtol=3e-3, atol=2e-3)
    ld, am = ti.DeviceBuffer(M * N * 4), ti.DeviceBuffer(M * ti.ARGMAX_SLOTS * 8)
    am.zero()
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out, ep.argmax = ti.EPI_LOGITS_ARGMAX, N, ld.ptr, am.ptr
    tiles, scales = ti.wpack_host(w, 4)
    run(ti, dev(ti, tiles), dev(ti, scales), xd, M, N, K, ep)
    logits = ld.download(f32, (M, N))
    keys = am.download(np.uint64, (M, ti.ARGMAX_SLOTS)).max(axis=1)
    np.testing.assert_array_equal((0xFFFFFFFF - (keys & 0xFFFFFFFF)).astype(np.int64), np.argmax(logits, axis=1))
    np.testing.assert_allclose(logits, xa @ wf.astype(np.float64), rtol=1e-4, atol=1e-4)


def test_splitk_repeat_is_deterministic(ti, oracle, splitk_ws):
    """The last arriver sums the k-slices in slice order: repeated calls give identical bits."""
    M, K, N = 128, 11008, 4096
    assert tile_plan(ti, M, N, K)[2] > 1
    rng = np.random.RandomState(11)
    w = (rng.standard_normal((K, N)) * 0.03).astype(f32)
    x = rng.standard_normal((M, K)).astype(f16)
    tiles, scales = ti.wpack_host(w, 4)
    td, sd, xd = dev(ti, tiles), dev(ti, scales), dev(ti, x)
    outs = []
    for _ in range(3):
        yd = ti.DeviceBuffer(M * N * 4)
        ep = ti.Epilogue()
        ep.kind, ep.ldo, ep.out = ti.EPI_STORE_F32, N, yd.ptr
        run(ti, td, sd, xd, M, N, K, ep, splitk_ws)
        outs.append(yd.download(f32, (M, N)))
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    assert np.array_equal(outs[0].view(np.uint32), outs[2].view(np.uint32))
    wf = deq(oracle, w, 4)
    xa = x.astype(f32)
    assert_close_dot(outs[0], xa.astype(np.float64) @ wf.astype(np.float64), xa, wf)


@pytest.mark.parametrize("splitk", [False, True])
def test_batched_resid_silu_logits(ti, oracle, splitk_ws, splitk):
    M, K = 57, 2048
    ws = splitk_ws if splitk else None
    rng = np.random.RandomState(5)
    x = rng.standard_normal((M, K)).astype(f16)
    xd, xa = dev(ti, x), x.astype(np.float64)
    # residual add in place
    N = 512
    w = (rng.standard_normal((K, N)) * 0.03).astype(f32)
    tiles, scales = ti.wpack_host(w, 4)
    r = rng.standard_normal((M, N)).astype(f32)
    rd = dev(ti, r)
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_RESID_F32, N, rd.ptr
    run(ti, dev(ti, tiles), dev(ti, scales), xd, M, N, K, ep, ws)
    wf = deq(oracle, w, 4)
    assert_close_dot(rd.download(f32, (M, N)) - r, xa @ wf.astype(np.float64), x.astype(f32), wf, rel=5e-5)
    # SiLU(gate) * up, gate/up interleaved 8 rows each per tile
    I = 200
    g = (rng.standard_normal((K, I)) * 0.05).astype(f32)
    u = (rng.standard_normal((K, I)) * 0.05).astype(f32)
    tiles, scales = ti.wpack_host(g, 4, n_total=2 * I, row_map=ti.ROWS_INTERLEAVE8, row_offset=0)
    ti.wpack_host(u, 4, n_total=2 * I, row_map=ti.ROWS_INTERLEAVE8, row_offset=8, tiles=tiles, scales=scales)
    yd = ti.DeviceBuffer(M * I * 2)
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_SILU_MUL_F16, I, yd.ptr
    run(ti, dev(ti, tiles), dev(ti, scales), xd, M, 2 * I, K, ep, ws)
    gg, uu = xa @ deq(oracle, g, 4).astype(np.float64), xa @ deq(oracle, u, 4).astype(np.float64)
    np.testing.assert_allclose(yd.download(f16, (M, I)).astype(np.float64), uu * (gg / (1 + np.exp(-gg))),
                               rtol=3e-3, atol=2e-3)
    # logits + argmax (slots per row), step counter
    V = 3008
    w = (rng.standard_normal((K, V)) * 0.05).astype(f32)
    tiles, scales = ti.wpack_host(w, 4)
    ld, am = ti.DeviceBuffer(M * V * 4), ti.DeviceBuffer(M * ti.ARGMAX_SLOTS * 8)
    am.zero()
    ctr = dev(ti, np.array([3], np.int32))
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out, ep.argmax, ep.step_ctr, ep.advance = ti.EPI_LOGITS_ARGMAX, V, ld.ptr, am.ptr, ctr.ptr, 2
    run(ti, dev(ti, tiles), dev(ti, scales), xd, M, V, K, ep, ws)
    logits = ld.download(f32, (M, V))
    keys = am.download(np.uint64, (M, ti.ARGMAX_SLOTS)).max(axis=1)
    np.testing.assert_array_equal((0xFFFFFFFF - (keys & 0xFFFFFFFF)).astype(np.int64), np.argmax(logits, axis=1))
    assert ctr.download(np.int32, (1,))[0] == 5
    np.testing.assert_allclose(logits, xa @ deq(oracle, w, 4).astype(np.float64), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("splitk", [False, True])
@pytest.mark.parametrize("hd,nh,nkv", [(128, 4, 4), (64, 8, 2)])
def test_batched_qkv_rope_kv_append(ti, oracle, splitk_ws, hd, nh, nkv, splitk):
    M, H, max_seq, theta = 45, 512, 40, 10000.0
    qd, kvd = nh * hd, nkv * hd
    N = qd + 2 * kvd
    rng = np.random.RandomState(hd + nh)
    ws = [(rng.standard_normal((H, n)) * 0.05).astype(f32) for n in (qd, kvd, kvd)]
    tiles = scales = None
    for w, off in zip(ws, (0, qd, qd + kvd)):
        tiles, scales = ti.wpack_host(w, 4, n_total=N, row_offset=off, tiles=tiles, scales=scales)
    x = rng.standard_normal((M, H)).astype(f16)
    pos = rng.randint(0, max_seq, size=M).astype(np.int32)
    cs = ti.rope_table(np.arange(max_seq, dtype=f32), hd, theta)
    qbuf = ti.DeviceBuffer(M * qd * 4)
    stride = nkv * max_seq * hd
    kc, vc = ti.DeviceBuffer(M * stride * 2), ti.DeviceBuffer(M * stride * 2)
    kc.zero(), vc.zero()
    posd, csd = dev(ti, pos), dev(ti, cs)
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_QKV_ROPE_KV, qd, qbuf.ptr
    ep.q_dim, ep.kv_dim, ep.head_dim, ep.max_seq = qd, kvd, hd, max_seq
    ep.pos, ep.rope_cs, ep.k_cache, ep.v_cache, ep.kv_stream_stride = posd.ptr, csd.ptr, kc.ptr, vc.ptr, stride
    run(ti, dev(ti, tiles), dev(ti, scales), dev(ti, x), M, N, H, ep, splitk_ws if splitk else None)
    q, k, v = (x.astype(np.float64) @ deq(oracle, w, 4).astype(np.float64) for w in ws)
    kcache = kc.download(f16, (M, nkv, max_seq, hd)).astype(f32)
    vcache = vc.download(f16, (M, nkv, max_seq, hd)).astype(f32)
    qgot = qbuf.download(f32, (M, qd))
    for m in range(M):
        p = np.array([pos[m]], f32)
        qr = oracle.apply_rope(q[m].astype(f32).reshape(1, nh, 1, hd), p, theta).reshape(-1)
        kr = oracle.apply_rope(k[m].astype(f32).reshape(1, nkv, 1, hd), p, theta).reshape(nkv, hd)
        np.testing.assert_allclose(qgot[m], qr, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(kcache[m, :, pos[m]], kr, rtol=2e-3, atol=2e-3)
        np.testing.assert_allclose(vcache[m, :, pos[m]], v[m].reshape(nkv, hd), rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("K", [2048, 11008, 16384, 20480])
def test_rmsnorm_f16_row_lengths(ti, oracle, K):
    """ti_rmsnorm_f16 at row lengths of 1 to 5 pieces of 8 floats per thread (the hidden sizes of
    the served models and past them) against the oracle's rms_norm."""
    M = 3
    rng = np.random.RandomState(K)
    x = (rng.standard_normal((M, K)) * 2).astype(f32)
    nw = (1 + 0.1 * rng.standard_normal(K)).astype(f32)
    xd, nwd = dev(ti, x), dev(ti, nw)
    yd = ti.DeviceBuffer(M * K * 2)
    ti.check(ti.lib().ti_rmsnorm_f16(xd.ptr, K, nwd.ptr, 1e-5, yd.ptr, K, M, K, None))
    ti.sync()
    ref = oracle.rms_norm(x, nw)
    np.testing.assert_allclose(yd.download(f16, (M, K)).astype(f32), ref.astype(f16).astype(f32), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("K", [4096, 8192])
def test_rmsnorm_f16_matches_fused_prologue(ti, oracle, K):
    """ti_rmsnorm_f16 rows fed to the fused kernel == its own rms_norm prologue (same arithmetic)."""
    M, N = 2, 256
    rng = np.random.RandomState(9)
    x = (rng.standard_normal((M, K)) * 2).astype(f32)
    nw = (1 + 0.1 * rng.standard_normal(K)).astype(f32)
    xd, nwd = dev(ti, x), dev(ti, nw)
    yd = ti.DeviceBuffer(M * K * 2)
    ti.check(ti.lib().ti_rmsnorm_f16(xd.ptr, K, nwd.ptr, 1e-5, yd.ptr, K, M, K, None))
    ti.sync()
    y = yd.download(f16, (M, K)).astype(f32)
    ref = oracle.rms_norm(x, nw)
    np.testing.assert_allclose(y, ref.astype(f16).astype(f32), rtol=1e-3, atol=1e-3)
    # the fused path's staged rows are the same fp16 values: identical GEMM results
    w = (rng.standard_normal((K, N)) * 0.03).astype(f32)
    tiles, scales = ti.wpack_host(w, 4)
    td, sd = dev(ti, tiles), dev(ti, scales)
    L = ti.lib()
    outs = []
    for xk, src, norm in ((ti.X_F32_RMSNORM, xd, nwd), (ti.X_F16, yd, None)):
        od = ti.DeviceBuffer(M * N * 4)
        ep = ti.Epilogue()
        ep.kind, ep.ldo, ep.out = ti.EPI_STORE_F32, N, od.ptr
        ti.check(L.ti_gemm_wq_a16(td.ptr, sd.ptr, 4, src.ptr, xk, K, norm.ptr if norm else None, 1e-5, M, N, K,
                                  C.byref(ep), None))
        ti.sync()
        outs.append(od.download(f32, (M, N)))
    np.testing.assert_array_equal(outs[0], outs[1])


# ------------------------------------------------------- fragment-packed operands (M > 16)
def test_packed_operands_match_row_major(ti, oracle):
    """TI_X_F16_PACKED: rms_norm prep, GEMM input, SiLU*up output and attention output in the
    batched-rows kernel's fragment order give the bit-identical numbers of the row-major forms
    (the same arithmetic; only addresses differ)."""
    L = ti.lib()
    rng = np.random.RandomState(11)
    M, K, N = 45, 1152, 512
    x32 = rng.standard_normal((M, K)).astype(f32)
    w = (rng.standard_normal(K) * 0.1 + 1).astype(f32)
    xd, wd = dev(ti, x32), dev(ti, w)
    Mp = (M + 15) // 16 * 16
    rm, pk = ti.DeviceBuffer(M * K * 2), ti.DeviceBuffer(Mp * K * 2)
    ti.check(L.ti_rmsnorm_f16(xd.ptr, K, wd.ptr, 1e-5, rm.ptr, K, M, K, None))
    ti.check(L.ti_rmsnorm_f16_packed(xd.ptr, K, wd.ptr, 1e-5, pk.ptr, M, K, None))
    ti.sync()
    rows = rm.download(np.uint16, (M, K))
    np.testing.assert_array_equal(ti.unpack_rows(pk.download(np.uint16, Mp * K), M, K), rows)
    # GEMM on both forms: store, and SiLU*up written packed
    wt = (rng.standard_normal((K, N)) * 0.03).astype(f32)
    tiles, scales = ti.wpack_host(wt, 4)
    td, sd = dev(ti, tiles), dev(ti, scales)
    outs = []
    for xk, xb in ((ti.X_F16, rm), (ti.X_F16_PACKED, pk)):
        yd = ti.DeviceBuffer(M * N * 4)
        ep = ti.Epilogue()
        ep.kind, ep.ldo, ep.out = ti.EPI_STORE_F32, N, yd.ptr
        ti.check(L.ti_gemm_wq_a16(td.ptr, sd.ptr, 4, xb.ptr, xk, K, None, 1e-5, M, N, K, C.byref(ep), None))
        ti.sync()
        outs.append(yd.download(f32, (M, N)))
    np.testing.assert_array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    I = 256
    g = (rng.standard_normal((K, I)) * 0.05).astype(f32)
    u = (rng.standard_normal((K, I)) * 0.05).astype(f32)
    tg, sg = ti.wpack_host(g, 4, n_total=2 * I, row_map=ti.ROWS_INTERLEAVE8, row_offset=0)
    ti.wpack_host(u, 4, n_total=2 * I, row_map=ti.ROWS_INTERLEAVE8, row_offset=8, tiles=tg, scales=sg)
    tgd, sgd = dev(ti, tg), dev(ti, sg)        # (held: a temporary's buffer would be freed before the launch)
    acts = []
    for packed in (0, 1):
        yd = ti.DeviceBuffer(Mp * I * 2)
        ep = ti.Epilogue()
        ep.kind, ep.ldo, ep.out, ep.out_packed = ti.EPI_SILU_MUL_F16, I, yd.ptr, packed
        ti.check(L.ti_gemm_wq_a16(tgd.ptr, sgd.ptr, 4, pk.ptr, ti.X_F16_PACKED, K, None, 1e-5, M, 2 * I, K,
                                  C.byref(ep), None))
        ti.sync()
        a = yd.download(np.uint16, Mp * I)
        acts.append(ti.unpack_rows(a, M, I) if packed else a[: M * I].reshape(M, I))
    np.testing.assert_array_equal(acts[0], acts[1])
    # attention output, both layouts
    heads, kvh, hd, max_seq = 4, 2, 64, 48
    q = rng.standard_normal((M, heads * hd)).astype(f32)
    kc = (rng.standard_normal((M, kvh, max_seq, hd)) * 0.5).astype(np.float16)
    vc = (rng.standard_normal((M, kvh, max_seq, hd)) * 0.5).astype(np.float16)
    pos = rng.randint(0, max_seq, size=M).astype(np.int32)
    qd_, kd, vd, pd = dev(ti, q), dev(ti, kc), dev(ti, vc), dev(ti, pos)
    ws = ti.DeviceBuffer(L.ti_attn_workspace_bytes(M, heads, hd, 4))
    ws.zero()
    o_rm, o_pk = ti.DeviceBuffer(M * heads * hd * 2), ti.DeviceBuffer(Mp * heads * hd * 2)
    stride = kvh * max_seq * hd
    ti.check(L.ti_attn_decode(qd_.ptr, kd.ptr, vd.ptr, stride, max_seq, pd.ptr, M, heads, kvh, hd, 4, ws.ptr,
                              o_rm.ptr, None))
    ti.check(L.ti_attn_decode_packed(qd_.ptr, kd.ptr, vd.ptr, stride, max_seq, pd.ptr, M, heads, kvh, hd, 4, ws.ptr,
                                     o_pk.ptr, None))
    ti.sync()
    np.testing.assert_array_equal(ti.unpack_rows(o_pk.download(np.uint16, Mp * heads * hd), M, heads * hd),
                                  o_rm.download(np.uint16, (M, heads * hd)))


# ------------------------------------------------------- batched fold (17..64 rows)
@pytest.mark.parametrize("M", [17, 32, 45, 64])
@pytest.mark.parametrize("packed", [1, 0])
def test_batched_fold_producer_consumer(ti, oracle, M, packed):
    """The batched fold (ti_hip.h TI_FOLD_SS_ROWS): a batched-rows residual epilogue also writes
    fp16(h * nw) (fragment-packed or row-major) and per-column-group sums of h^2 per row; the
    next call takes those rows with ss_in and normalises behind its GEMM.  Against the rms_norm
    prep path (ti_rmsnorm_f16[_packed] + the same GEMM): the two differ only in where the fp16
    rounding of the normalised row happens (rtol 4e-3 on the outputs)."""
    L = ti.lib()
    K, H, N = 1152, 1024, 768 if packed else 25600   # consumer: rows kernel (packed) / tile kernel
    assert L.ti_gemm_packed_rows_for(4, M, N, H) == packed
    rng = np.random.RandomState(M + 100 * packed)
    act = rng.standard_normal((M, K)).astype(f16)
    wo = (rng.standard_normal((K, H)) * 0.03).astype(f32)
    h0 = rng.standard_normal((M, H)).astype(f32)
    nw = (1 + 0.1 * rng.standard_normal(H)).astype(f32)
    to, so = ti.wpack_host(wo, 4)
    tod, sod, actd, nwd = dev(ti, to), dev(ti, so), dev(ti, ti.pack_rows(act)), dev(ti, nw)
    n_ss = L.ti_gemm_fold_partials(4, M, H, K)
    assert 1 <= n_ss <= 4096
    Mp = (M + 15) // 16 * 16
    hd, fx, ss = dev(ti, h0), ti.DeviceBuffer(Mp * H * 2), ti.DeviceBuffer(n_ss * 64 * 4)
    fx.zero()
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_RESID_F32, H, hd.ptr
    ep.fold_w, ep.fold_x, ep.fold_ss, ep.fold_packed = nwd.ptr, fx.ptr, ss.ptr, packed
    ti.check(L.ti_gemm_wq_a16(tod.ptr, sod.ptr, 4, actd.ptr, ti.X_F16_PACKED, K, None, 1e-5, M, H, K, C.byref(ep), None))
    ti.sync()
    h1 = hd.download(f32, (M, H))
    assert_close_dot(h1 - h0, act.astype(np.float64) @ deq(oracle, wo, 4).astype(np.float64), act.astype(f32),
                     deq(oracle, wo, 4), rel=5e-5)
    # the folded outputs: exactly fp16(h * nw) of the stored h, and the row sums of h^2
    fxr = fx.download(np.uint16, Mp * H)
    fxr = ti.unpack_rows(fxr, M, H) if packed else fxr[: M * H].reshape(M, H)
    np.testing.assert_array_equal(fxr, (h1 * nw).astype(f16).view(np.uint16))
    ssr = ss.download(f32, (n_ss, 64))[:, :M].sum(axis=0)
    np.testing.assert_allclose(ssr, (h1.astype(np.float64) ** 2).sum(axis=1), rtol=1e-5)
    # consumer: folded rows + ss_in against the rms_norm prep of the same h
    w2 = (rng.standard_normal((H, N)) * 0.03).astype(f32)
    t2, s2 = ti.wpack_host(w2, 4)
    t2d, s2d = dev(ti, t2), dev(ti, s2)
    outs = []
    for fold in (True, False):
        yd = ti.DeviceBuffer(M * N * 4)
        ep = ti.Epilogue()
        ep.kind, ep.ldo, ep.out = ti.EPI_STORE_F32, N, yd.ptr
        xk = ti.X_F16_PACKED if packed else ti.X_F16
        if fold:
            ep.ss_in, ep.n_ss = ss.ptr, n_ss
            src = fx
        else:
            src = ti.DeviceBuffer(Mp * H * 2)
            fn = L.ti_rmsnorm_f16_packed if packed else None
            if packed:
                ti.check(fn(hd.ptr, H, nwd.ptr, 1e-5, src.ptr, M, H, None))
            else:
                ti.check(L.ti_rmsnorm_f16(hd.ptr, H, nwd.ptr, 1e-5, src.ptr, H, M, H, None))
        ti.check(L.ti_gemm_wq_a16(t2d.ptr, s2d.ptr, 4, src.ptr, xk, H, None, 1e-5, M, N, H, C.byref(ep), None))
        ti.sync()
        outs.append(yd.download(f32, (M, N)))
    rms = np.sqrt((h1.astype(np.float64) ** 2).mean(axis=1) + 1e-5)
    ref = ((h1 / rms[:, None]) * nw).astype(np.float64) @ deq(oracle, w2, 4).astype(np.float64)
    scale = np.abs(ref).max()
    assert np.abs(outs[0] - ref).max() <= 4e-3 * scale
    assert np.abs(outs[0] - outs[1]).max() <= 4e-3 * scale
    # a repeated folded call gives the same bits (fixed-order partial sums)
    yd = ti.DeviceBuffer(M * N * 4)
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out, ep.ss_in, ep.n_ss = ti.EPI_STORE_F32, N, yd.ptr, ss.ptr, n_ss
    ti.check(L.ti_gemm_wq_a16(t2d.ptr, s2d.ptr, 4, fx.ptr, ti.X_F16_PACKED if packed else ti.X_F16, H, None, 1e-5, M,
                              N, H, C.byref(ep), None))
    ti.sync()
    np.testing.assert_array_equal(yd.download(f32, (M, N)).view(np.uint32), outs[0].view(np.uint32))


def test_batched_fold_refuses_other_kernels(ti):
    """fold_x at M > 1 needs packed x (the batched-rows kernel); a folded input needs M <= 64."""
    L = ti.lib()
    M, K, N = 40, 1152, 512
    buf = ti.DeviceBuffer(128 * 4096 * 4)
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out = ti.EPI_RESID_F32, N, buf.ptr
    ep.fold_w, ep.fold_x, ep.fold_ss = buf.ptr, buf.ptr, buf.ptr
    tiles, scales = ti.wpack_host(np.zeros((K, N), f32), 4)
    td, sd = dev(ti, tiles), dev(ti, scales)
    assert L.ti_gemm_wq_a16(td.ptr, sd.ptr, 4, buf.ptr, ti.X_F16, K, None, 1e-5, M, N, K, C.byref(ep), None) != 0
    ep = ti.Epilogue()
    ep.kind, ep.ldo, ep.out, ep.ss_in, ep.n_ss = ti.EPI_STORE_F32, N, buf.ptr, buf.ptr, 4
    assert L.ti_gemm_wq_a16(td.ptr, sd.ptr, 4, buf.ptr, ti.X_F16, K, None, 1e-5, 100, N, K, C.byref(ep), None) != 0
