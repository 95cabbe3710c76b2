"""Prefill attention on MFMA (ti_attn_prefill, prefill_attn.hip): the rows of a prompt chunk
attend causally to their own stream's cache (forward_pass, inference_engine.cpp:1429-1491 ->
multi_head_attention, tensor_engine.cpp:1149-1252).

Every kernel the call can choose (ti_attn_prefill_set_kernel: per-wave, shared-K/V in 4- and
8-wave workgroups) is checked at every shape.  Against the oracle's multi_head_attention per row (the bar of test_gpu_kernels.py's attention
tests: fp16 output, rtol = atol = 4e-3) and against ti_attn_decode with stream stride 0 (the
decode kernel the engine used for prefill before; same bar).  Cache rows past the chunk's last
position hold NaN, as unwritten memory may: they must not reach any output."""
from __future__ import annotations

import numpy as np
import pytest

from test_gpu_kernels import dev

pytestmark = pytest.mark.gpu
f16, f32 = np.float16, np.float32


def _case(ti, M, nh, nkv, hd, pos, max_seq, seed):
    rng = np.random.RandomState(seed)
    kc = rng.standard_normal((nkv, max_seq, hd)).astype(f16)
    vc = rng.standard_normal((nkv, max_seq, hd)).astype(f16)
    top = int(pos.max())
    kc[:, top + 1:] = np.nan
    vc[:, top + 1:] = np.nan
    q = rng.standard_normal((M, nh * hd)).astype(f32)
    kd, vd, qd_, pd = dev(ti, kc), dev(ti, vc), dev(ti, q), dev(ti, pos)
    L = ti.lib()
    out = ti.DeviceBuffer(M * nh * hd * 2)
    ti.check(L.ti_attn_prefill(qd_.ptr, kd.ptr, vd.ptr, max_seq, pd.ptr, M, nh, nkv, hd, out.ptr, None))
    ti.sync()
    got = out.download(f16, (M, nh * hd)).astype(f32)
    if nh // nkv > 8:   # the decode kernel serves groups up to 8: the oracle alone is the reference
        return q, kc, vc, got, None
    ref = ti.DeviceBuffer(M * nh * hd * 2)
    ws = ti.DeviceBuffer(L.ti_attn_workspace_bytes(M, nh, hd, 4))
    ws.zero()
    ti.check(L.ti_attn_decode(qd_.ptr, kd.ptr, vd.ptr, 0, max_seq, pd.ptr, M, nh, nkv, hd, 4, ws.ptr, ref.ptr, None))
    ti.sync()
    return q, kc, vc, got, ref.download(f16, (M, nh * hd)).astype(f32)


@pytest.fixture(params=[0, 1, 2, 3], ids=["auto", "per_wave", "shared4", "shared8"])
def kernel(request, ti):
    """ti_attn_prefill_set_kernel: the automatic choice, the per-wave kernel, and the shared-K/V
    kernel with 4- and 8-wave workgroups forced at any grid size (head_dim 128; other head_dims
    take the per-wave kernel)."""
    L = ti.lib()
    assert L.ti_attn_prefill_set_kernel(request.param) == 0
    yield request.param
    assert L.ti_attn_prefill_set_kernel(0) == request.param


@pytest.mark.parametrize("M,nh,nkv,hd,start,max_seq", [
    (1, 4, 4, 128, 0, 16),          # one row, one key
    (37, 4, 4, 128, 0, 64),         # partial 16-row block
    (64, 8, 2, 64, 5, 80),          # GQA 4, hd 64, start past 0
    (300, 8, 1, 128, 100, 512),     # GQA 8, a cache prefix before the chunk
    (129, 8, 4, 64, 0, 129),        # prefix ends at max_seq - 1
    (77, 32, 2, 128, 3, 96),        # GQA 16 (one row per wave), a partial last block
    (200, 8, 8, 128, 1000, 1200),   # MHA, long prefix before a chunk whose blocks straddle 16
])
def test_prefill_attention_vs_oracle(ti, oracle, kernel, M, nh, nkv, hd, start, max_seq):
    if hd != 128 and kernel > 1:
        pytest.skip("the shared-K/V kernel is head_dim 128 only")
    pos = (start + np.arange(M)).astype(np.int32)
    q, kc, vc, got, dec = _case(ti, M, nh, nkv, hd, pos, max_seq, seed=M + nh + hd)
    assert np.all(np.isfinite(got))
    grp = nh // nkv
    for m in list(range(0, M, max(1, M // 12))) + [M - 1]:
        S = int(pos[m]) + 1
        kx = np.repeat(kc[:, :S].astype(f32).transpose(1, 0, 2), grp, axis=1).reshape(1, S, nh * hd)
        vx = np.repeat(vc[:, :S].astype(f32).transpose(1, 0, 2), grp, axis=1).reshape(1, S, nh * hd)
        ref = oracle.multi_head_attention(q[m].reshape(1, 1, -1), kx, vx, nh).reshape(-1)
        np.testing.assert_allclose(got[m], ref, rtol=4e-3, atol=4e-3, err_msg=f"row {m}")
    if dec is not None:
        np.testing.assert_allclose(got, dec, rtol=4e-3, atol=4e-3)


@pytest.mark.parametrize("hd", [64, 128])
def test_prefill_attention_ragged_positions(ti, kernel, hd):
    """Positions in any order and with gaps (each row's own causal limit, blocks of mixed length)
    and the 7B chunk shape, against the decode kernel."""
    if hd != 128 and kernel > 1:
        pytest.skip("the shared-K/V kernel is head_dim 128 only")
    rng = np.random.RandomState(hd)
    pos = rng.permutation(900)[:333].astype(np.int32)
    _, _, _, got, dec = _case(ti, 333, 8, 2, hd, pos, 1024, seed=hd + 1)
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(got, dec, rtol=4e-3, atol=4e-3)


def test_prefill_attention_7b_chunk(ti):
    pos = np.arange(512, dtype=np.int32)
    _, _, _, got, dec = _case(ti, 512, 32, 32, 128, pos, 2048, seed=7)
    np.testing.assert_allclose(got, dec, rtol=4e-3, atol=4e-3)


@pytest.mark.parametrize("hd", [64, 128])
def test_prefill_attention_chunk_beyond_one_wave_per_simd(ti, hd):
    """A chunk with more waves than the chip has SIMDs (1024 rows x 32 heads = 2048 waves) takes the
    3-deep K / V ring (two waves per SIMD); the chunks above take the deep ring (ti_attn_prefill)."""
    pos = np.arange(1024, dtype=np.int32)
    _, _, _, got, dec = _case(ti, 1024, 32, 32, hd, pos, 1024, seed=hd + 3)
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(got, dec, rtol=4e-3, atol=4e-3)


def test_prefill_attention_set_kernel_rejects_bad_modes(ti):
    L = ti.lib()
    assert L.ti_attn_prefill_set_kernel(4) == -1
    assert L.ti_attn_prefill_set_kernel(-1) == -1
    assert L.ti_attn_prefill_set_kernel(0) == 0


def test_prefill_attention_rejects_bad_sizes(ti):
    L = ti.lib()
    assert L.ti_attn_prefill(1, 1, 1, 16, 1, 0, 4, 4, 128, 1, None) != 0
    assert L.ti_attn_prefill(1, 1, 1, 16, 1, 4, 6, 4, 128, 1, None) != 0
    assert L.ti_attn_prefill(1, 1, 1, 16, 1, 4, 4, 4, 96, 1, None) != 0
