"""CPU-side checks of the product library: it loads, exports every symbol the C headers
declare, host-side argument checks fail with TI_ERR_ARG without touching a GPU, and the
host weight packer is bit-identical to the oracle's group quantizer."""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np
import pytest

import turboinfer_amd as T
from conftest import ROOT
from packing import unpack_tiles


def header_functions(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\**\s+\**(ti_[a-z0-9_]+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(T.LIB_PATH):
        T.build()
    return T.lib()


def test_gemm_max_rows(L):
    # fused kernel: rows while the LDS image fits; int4 + fp16 rows: the batched-rows kernel
    assert L.ti_gemm_max_rows(4, T.X_F16, 4096, 4096) == T.GEMM_MAX_ROWS
    assert L.ti_gemm_max_rows(4, T.X_F16, 4096, 11008) == T.GEMM_MAX_ROWS
    assert L.ti_gemm_max_rows(4, T.X_F32_RMSNORM, 12288, 4096) == 2
    assert L.ti_gemm_max_rows(8, T.X_F32_RMSNORM, 12288, 4096) == 16
    assert 1 <= L.ti_gemm_max_rows(8, T.X_F16, 4096, 11008) < 16
    assert L.ti_gemm_max_rows(4, T.X_F16, 8, 4096) == 0


def test_exports_every_declared_symbol(L):
    declared = header_functions(os.path.join(ROOT, "include", "ti_hip.h")) + \
        header_functions(os.path.join(ROOT, "include", "ti_engine.h"))
    assert len(declared) >= 50
    missing = [f for f in declared if not hasattr(L, f)]
    assert not missing, missing
    assert sorted(declared) == sorted(T.EXPORTED)


def test_epilogue_mirror_matches_abi(L):
    # the ctypes mirror of ti_epilogue must have the library's size (trailing fields included)
    assert L.ti_epilogue_bytes() == C.sizeof(T.Epilogue)


def test_argument_errors_are_reported_without_launch(L):
    ep = T.Epilogue()
    ep.kind = T.EPI_STORE_F32
    ep.ldo = 16
    ep.out = 1234
    # M out of range
    rc = L.ti_gemm_wq_a16(1, 1, 4, 1, T.X_F16, 128, None, 1e-5, 0, 16, 128, C.byref(ep), None)
    assert rc == 1 and b"M must be" in L.ti_last_error()
    # K not a multiple of 128
    rc = L.ti_gemm_wq_a16(1, 1, 4, 1, T.X_F16, 129, None, 1e-5, 1, 16, 129, C.byref(ep), None)
    assert rc == 1 and b"K %" in L.ti_last_error()
    # bad bits
    rc = L.ti_gemm_wq_a16(1, 1, 3, 1, T.X_F16, 128, None, 1e-5, 1, 16, 128, C.byref(ep), None)
    assert rc == 1
    # rows beyond the fused kernel need int4 + fp16 rows (the batched-rows kernel)
    rc = L.ti_gemm_wq_a16(1, 1, 4, 1, T.X_F32_RMSNORM, 11008, 1, 1e-5, 12, 16, 11008, C.byref(ep), None)
    assert rc == 3 and b"batched-rows" in L.ti_last_error()
    rc = L.ti_gemm_wq_a16(1, 1, 8, 1, T.X_F16, 4096, None, 1e-5, 20, 16, 4096, C.byref(ep), None)
    assert rc == 3
    rc = L.ti_gemm_wq_a16(1, 1, 4, 1, T.X_F16, 4096, None, 1e-5, T.GEMM_MAX_ROWS + 1, 16, 4096, C.byref(ep), None)
    assert rc == 1 and b"M must be" in L.ti_last_error()
    rc = L.ti_rmsnorm_f16(1, 100, 1, 1e-5, 1, 128, 2, 128, None)
    assert rc == 1
    # folded rms_norm input: one row, ss partials required; fold producer: one row
    rc = L.ti_gemm_wq_a16(1, 1, 4, 1, T.X_F16_FOLDED, 4096, None, 1e-5, 2, 16, 4096, C.byref(ep), None)
    assert rc == 1 and b"TI_X_F16_FOLDED" in L.ti_last_error()
    rc = L.ti_gemm_wq_a16(1, 1, 4, 1, T.X_F16_FOLDED, 4096, None, 1e-5, 1, 16, 4096, C.byref(ep), None)
    assert rc == 1 and b"TI_X_F16_FOLDED" in L.ti_last_error()
    fe = T.Epilogue()
    fe.kind, fe.ldo, fe.out, fe.fold_x = T.EPI_RESID_F32, 16, 1234, 1234
    rc = L.ti_gemm_wq_a16(1, 1, 4, 1, T.X_F16, 4096, None, 1e-5, 1, 16, 4096, C.byref(fe), None)
    assert rc == 1 and b"fold_x" in L.ti_last_error()
    assert L.ti_gemm_grid(1, 4096, 4096) >= 1 and L.ti_gemm_grid(1, 4096, 4096) <= 256
    assert L.ti_gemm_grid(0, 4096, 4096) == 0
    # batched fold: producer partials for the configs[3] / [4] O and down shapes; none outside 17..64
    # int4 rows; a batched fold_x needs packed x, a batched folded input at most 64 rows
    for M, N, K in [(64, 4096, 4096), (64, 4096, 11008), (32, 4096, 4096), (32, 4096, 14336), (17, 4096, 4096)]:
        assert 1 <= L.ti_gemm_fold_partials(4, M, N, K) <= 4096
    assert L.ti_gemm_fold_partials(4, 16, 4096, 4096) == 0 and L.ti_gemm_fold_partials(4, 65, 4096, 4096) == 0
    assert L.ti_gemm_fold_partials(8, 32, 4096, 4096) == 0
    rc = L.ti_gemm_wq_a16(1, 1, 4, 1, T.X_F16, 4096, None, 1e-5, 32, 16, 4096, C.byref(fe), None)
    assert rc == 1 and b"batched fold_x" in L.ti_last_error()
    be = T.Epilogue()
    be.kind, be.ldo, be.out, be.ss_in, be.n_ss = T.EPI_STORE_F32, 16, 1234, 1234, 8
    rc = L.ti_gemm_wq_a16(1, 1, 4, 1, T.X_F16, 4096, None, 1e-5, 100, 16, 4096, C.byref(be), None)
    assert rc == 1 and b"batched folded input" in L.ti_last_error()
    # attention head_dim unsupported
    rc = L.ti_attn_decode(1, 1, 1, 1 << 20, 16, 1, 1, 4, 4, 96, 1, 1, 1, None)
    assert rc == 3
    # GQA group not supported
    rc = L.ti_attn_decode(1, 1, 1, 1 << 20, 16, 1, 1, 12, 4, 128, 1, 1, 1, None)
    assert rc in (1, 3)


def test_engine_config_validation(L):
    cfg = T.EngineConfig(1000, 256, 2, 4, 4, 64, 512, 1e4, 1e-5, 4, 64, 1, 0, 0, 0)
    h = C.c_void_p()
    rc = L.ti_engine_create(C.byref(cfg), C.byref(h))
    assert rc != 0   # vocab 1000 not a multiple of 16 (or no device here)
    cfg = T.EngineConfig(1024, 256, 2, 6, 4, 64, 512, 1e4, 1e-5, 4, 64, 1, 0, 0, 0)
    assert L.ti_engine_create(C.byref(cfg), C.byref(h)) != 0  # heads % kv_heads
    # generate()'s stop token and the step counters need an engine
    assert L.ti_engine_set_stop(None, 2) == 1 and b"ti_engine_set_stop" in L.ti_last_error()
    assert L.ti_engine_counters(None, None, None) == 1


@pytest.mark.parametrize("bits", [4, 8, 16])
@pytest.mark.parametrize("scale_mode", [0, 1])
def test_host_packer_matches_oracle_quantizer(oracle, bits, scale_mode):
    if bits == 16 and scale_mode:
        pytest.skip("fp16 weights carry no scale")
    K, N = 256, 48
    w = (np.random.RandomState(7).standard_normal((K, N)) * 0.03).astype(np.float32)
    tiles, scales = T.wpack_host(w, bits, scale_mode=scale_mode)
    q, s = unpack_tiles(tiles, scales, bits, K, N)
    if bits == 16:
        np.testing.assert_array_equal(q.view(np.uint16), w.T.astype(np.float16).view(np.uint16))
        return
    qo, so = oracle.quantize_groups(w, bits, 128, scale_mode)
    np.testing.assert_array_equal(q, qo)
    np.testing.assert_array_equal(s, so)


def test_host_packer_fused_rows(oracle):
    """QKV concatenation and gate/up interleave-by-8 land each source column on its row."""
    K, I = 128, 32
    g = (np.random.RandomState(1).standard_normal((K, I)) * 0.05).astype(np.float32)
    u = (np.random.RandomState(2).standard_normal((K, I)) * 0.05).astype(np.float32)
    tiles, scales = T.wpack_host(g, 4, n_total=2 * I, row_map=T.ROWS_INTERLEAVE8, row_offset=0)
    T.wpack_host(u, 4, n_total=2 * I, row_map=T.ROWS_INTERLEAVE8, row_offset=8, tiles=tiles, scales=scales)
    q, s = unpack_tiles(tiles, scales, 4, K, 2 * I)
    qg, sg = oracle.quantize_groups(g, 4)
    qu, su = oracle.quantize_groups(u, 4)
    for c in range(I):
        rg = 16 * (c // 8) + c % 8
        np.testing.assert_array_equal(q[rg], qg[c])
        np.testing.assert_array_equal(q[rg + 8], qu[c])
        assert s[rg, 0] == sg[c, 0] and s[rg + 8, 0] == su[c, 0]


def test_int4_range_is_reference_symmetric(oracle):
    """INT4 values stay in [-7, 7] like quantize_to_int4's symmetric clamp (quantization.cpp:684-686)."""
    w = (np.random.RandomState(5).standard_normal((128, 16)) * 10).astype(np.float32)
    tiles, scales = T.wpack_host(w, 4)
    q, _ = unpack_tiles(tiles, scales, 4, 128, 16)
    assert q.min() >= -7 and q.max() <= 7 and q.min() == -7 or q.max() == 7


def test_wpack_q41_rounding_matches_ggml(L):
    """fp32 weights packed for an affine group-32 engine (ti_wpack_host, bits 4 | G32 | AFF)
    equal the packing of ggml's Q4_1 blocks of the same weights (gguf_oracle.quant_q4_1, the
    reference quantizer) through ti_wpack_q1_host: same rounding, same fp16 d and m."""
    import gguf_oracle as G
    K, N = 256, 48
    rng = np.random.RandomState(11)
    w = (rng.standard_normal((K, N)) * 0.05 + rng.uniform(-0.02, 0.02, (1, N))).astype(np.float32)
    w[32:64, 5] = 0.125                           # a constant block: d = 0
    bits = 4 | T.BITS_G32 | T.BITS_AFF
    tb, sb = L.ti_wpack_tile_bytes(bits, K, N), L.ti_wpack_scale_bytes(bits, K, N)
    assert sb == 2 * L.ti_wpack_scale_bytes(4 | T.BITS_G32, K, N)
    t1, s1 = np.zeros(tb, np.uint8), np.zeros(sb // 2, np.uint16)
    assert L.ti_wpack_host(w.ctypes.data, K, N, N, bits, T.SCALE_GROUP, 0, 0, t1.ctypes.data, s1.ctypes.data) == 0
    raw = np.frombuffer(G.quant_q4_1(np.ascontiguousarray(w.T)), np.uint8).reshape(N, K // 32, 20)
    d = raw[:, :, 0:2].copy().view(np.uint16)[..., 0].T.copy()
    m = raw[:, :, 2:4].copy().view(np.uint16)[..., 0].T.copy()
    qs = raw[:, :, 4:]
    q = np.concatenate([qs & 15, qs >> 4], axis=2).reshape(N, K).T.copy()   # [K][N], 0..15
    t2, s2 = np.zeros(tb, np.uint8), np.zeros(sb // 2, np.uint16)
    assert L.ti_wpack_q1_host(q.ctypes.data, d.ctypes.data, m.ctypes.data, K, N, N, 0, 0, t2.ctypes.data,
                              s2.ctypes.data) == 0
    assert np.array_equal(t1, t2) and np.array_equal(s1, s2)
