"""turboinfer_amd -- MI355X (gfx950) decode hot path of TurboInfer.

The product is the native library turboinfer_amd/lib/libturboinfer_amd.so:
  * the extern "C" kernel boundary   include/ti_hip.h    (HIP kernels for gfx950)
  * the extern "C" decode engine     include/ti_engine.h (device-resident decode loop)
  * the C++20 drop-in API            include/turboinfer/ (turboinfer::core / model / optimize)

This module is a thin ctypes binding of the two C headers for Python hosts (tests, bench).
It never falls back to a CPU implementation: if the library or a GPU is missing, calls fail
loudly with TiError.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# TI_LIB: an alternative in-tree build of the same library (A/B experiments)
LIB_PATH = os.environ.get("TI_LIB") or os.path.join(HERE, "lib", "libturboinfer_amd.so")

TI_OK = 0
X_F16, X_F32, X_F32_RMSNORM, X_F16_FOLDED, X_ATTN_SPLITS, X_F16_PACKED = 0, 1, 2, 3, 4, 5
ATTN_MAX_PART_SPLITS = 8           # TI_ATTN_MAX_PART_SPLITS (include/ti_hip.h)
EPI_STORE_F32, EPI_STORE_F16, EPI_RESID_F32, EPI_SILU_MUL_F16, EPI_QKV_ROPE_KV, EPI_LOGITS_ARGMAX = range(6)
ARGMAX_SLOTS = 32
GEMM_MAX_ROWS = 1024                # TI_GEMM_MAX_ROWS (include/ti_hip.h)
BITS_G32 = 32                       # TI_BITS_G32 (include/ti_hip.h): group-32 weights (GGUF Q4_0 / Q8_0)
BITS_AFF = 64                       # TI_BITS_AFF: affine group-32 int4 (GGUF Q4_1), with BITS_G32 | 4
SCALE_GROUP, SCALE_TENSOR, SCALE_UNIT = 0, 1, 2
ROWS_CONCAT, ROWS_INTERLEAVE8 = 0, 1
(W_Q, W_K, W_V, W_O, W_GATE, W_UP, W_DOWN, W_LM_HEAD, V_ATTN_NORM, V_FFN_NORM, V_OUT_NORM, E_EMBED) = range(12)


class TiError(RuntimeError):
    pass


class Epilogue(C.Structure):
    _fields_ = [("kind", C.c_int32), ("ldo", C.c_int32), ("out", C.c_void_p),
                ("q_dim", C.c_int32), ("kv_dim", C.c_int32), ("head_dim", C.c_int32), ("max_seq", C.c_int32),
                ("pos", C.c_void_p), ("rope_cs", C.c_void_p), ("k_cache", C.c_void_p), ("v_cache", C.c_void_p),
                ("kv_stream_stride", C.c_int64), ("argmax", C.c_void_p), ("step_ctr", C.c_void_p),
                ("advance", C.c_int32), ("n_ss", C.c_int32), ("ss_in", C.c_void_p),
                ("fold_w", C.c_void_p), ("fold_x", C.c_void_p), ("fold_ss", C.c_void_p), ("out_packed", C.c_int32),
                ("splitk_ws", C.c_void_p), ("splitk_bytes", C.c_int64), ("fold_packed", C.c_int32)]


class StepArgs(C.Structure):
    _fields_ = [("emb", C.c_void_p), ("h", C.c_void_p), ("hidden", C.c_int32), ("M", C.c_int32),
                ("vocab", C.c_int32), ("in_stride", C.c_int32), ("out_stride", C.c_int32),
                ("placeholder_first", C.c_int32), ("in_tokens", C.c_void_p), ("n_in", C.c_void_p),
                ("argmax", C.c_void_p), ("out_tokens", C.c_void_p), ("pos", C.c_void_p),
                ("base_pos", C.c_void_p), ("step_ctr", C.c_void_p), ("fold_w", C.c_void_p),
                ("fold_x", C.c_void_p), ("fold_ss", C.c_void_p)]


class EngineConfig(C.Structure):
    _fields_ = [("vocab", C.c_int32), ("hidden", C.c_int32), ("layers", C.c_int32), ("heads", C.c_int32),
                ("kv_heads", C.c_int32), ("head_dim", C.c_int32), ("inter", C.c_int32),
                ("rope_theta", C.c_float), ("eps", C.c_float), ("bits", C.c_int32), ("max_seq", C.c_int32),
                ("max_batch", C.c_int32), ("compat", C.c_int32), ("device", C.c_int32),
                ("attn_splits", C.c_int32)]


# Every symbol declared in include/ti_hip.h and include/ti_engine.h (checked by tests).
EXPORTED = [
    "ti_last_error", "ti_device_count", "ti_init", "ti_device_name", "ti_malloc", "ti_free", "ti_memcpy_h2d",
    "ti_memcpy_d2h", "ti_memcpy_d2d", "ti_memset", "ti_stream_create", "ti_stream_destroy", "ti_stream_sync",
    "ti_device_sync", "ti_event_create", "ti_event_destroy", "ti_event_record", "ti_event_elapsed_ms",
    "ti_wpack_tile_bytes", "ti_wpack_scale_bytes", "ti_wpack_host", "ti_wsynth_device", "ti_fill_uniform_f16",
    "ti_fill_uniform_f32", "ti_fill_kv_uniform", "ti_kv_copy_slots", "ti_gemm_wq_a16", "ti_gemm_lds_bytes", "ti_gemm_prepare",
    "ti_gemm_max_rows", "ti_gemm_packed_rows", "ti_gemm_packed_rows_for", "ti_gemm_tile_plan", "ti_rmsnorm_f16", "ti_rmsnorm_f16_packed", "ti_attn_decode_packed", "ti_attn_prefill", "ti_attn_prefill_set_kernel",
    "ti_attn_workspace_bytes", "ti_attn_decode", "ti_step_begin", "ti_matmul_f32", "ti_rms_norm_f32",
    "ti_rope_f32", "ti_silu_f32", "ti_relu_f32", "ti_add_f32", "ti_mul_f32", "ti_softmax_f32", "ti_attention_f32",
    "ti_argmax_f32", "ti_engine_create", "ti_engine_destroy", "ti_engine_get_stream", "ti_engine_memory", "ti_engine_set_tensor",
    "ti_engine_synth", "ti_engine_fill_kv", "ti_engine_generate", "ti_engine_step", "ti_engine_compat_step",
    "ti_engine_replay_prepare", "ti_engine_set_prefill", "ti_engine_replay_run", "ti_engine_sync", "ti_engine_last_tokens",
    "ti_engine_time_kernel", "ti_engine_stamp_steps", "ti_rope_table", "ti_sample_token", 
    "ti_gemm_grid", "ti_engine_set_fold",
    "ti_attn_decode_partials", "ti_sample_device", "ti_sample_step", "ti_engine_generate_sampled",
    "ti_engine_beam_search", "ti_engine_serve", 
    "ti_wpack_q_host", "ti_engine_set_tensor_q", "ti_sample_workspace_bytes", "ti_sample_device_ws",
    "ti_wpack_q1_host", "ti_engine_set_tensor_q1", "ti_epilogue_bytes",
    "ti_sample_step_ws", "ti_hbm_calibrate", "ti_gemm_kernel_name",
    "ti_gemm_fold_partials", "ti_engine_set_stop", "ti_engine_counters",
    "ti_qkv_attn_partials", "ti_qkv_attn_part_o_elems", "ti_qkv_attn_part_ml_elems", "ti_engine_set_qkv_attn",
    "ti_qkv_attn_xchg_bytes", "ti_qkv_attn_supported", "ti_qkv_attn_error_offset",
]

_lib = None


def build(jobs: int = 8) -> None:
    """Compile the native library in-tree (hipcc --offload-arch=gfx950)."""
    subprocess.run(["make", "-s", "-C", ROOT, f"-j{jobs}", "all"], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise TiError(f"native library missing: {LIB_PATH} (run `make` or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        vp, i32, i64, u64, f32, sz = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_float, C.c_size_t
        L.ti_last_error.restype = C.c_char_p
        L.ti_device_count.argtypes = [C.POINTER(C.c_int)]
        L.ti_init.argtypes = [i32]
        L.ti_device_name.argtypes = [i32, C.c_char_p, i32]
        L.ti_malloc.argtypes = [C.POINTER(vp), sz]
        L.ti_free.argtypes = [vp]
        for n in ("ti_memcpy_h2d", "ti_memcpy_d2h", "ti_memcpy_d2d"):
            getattr(L, n).argtypes = [vp, vp, sz, vp]
        L.ti_memset.argtypes = [vp, i32, sz, vp]
        L.ti_stream_sync.argtypes = [vp]
        L.ti_wpack_tile_bytes.argtypes = [i32, i32, i32]
        L.ti_wpack_tile_bytes.restype = sz
        L.ti_wpack_scale_bytes.argtypes = [i32, i32, i32]
        L.ti_wpack_scale_bytes.restype = sz
        L.ti_wpack_host.argtypes = [vp, i32, i32, i32, i32, i32, i32, i32, vp, vp]
        L.ti_wsynth_device.argtypes = [u64, C.c_uint32, i32, i32, i32, i32, i32, i32, vp, vp, vp]
        L.ti_fill_uniform_f16.argtypes = [u64, C.c_uint32, u64, f32, vp, vp]
        L.ti_fill_uniform_f32.argtypes = [u64, C.c_uint32, u64, f32, f32, vp, vp]
        L.ti_fill_kv_uniform.argtypes = [u64, C.c_uint32, i32, i32, i32, i32, vp, vp]
        L.ti_kv_copy_slots.argtypes = [vp, i32, C.c_int64, C.c_int64, i32, C.c_int64, C.c_int64, vp]
        L.ti_gemm_wq_a16.argtypes = [vp, vp, i32, vp, i32, i32, vp, f32, i32, i32, i32, C.POINTER(Epilogue), vp]
        L.ti_gemm_fold_partials.argtypes = [i32, i32, i32, i32]
        L.ti_gemm_lds_bytes.argtypes = [i32, i32, i32]
        L.ti_gemm_max_rows.argtypes = [i32, i32, i32, i32]
        L.ti_gemm_packed_rows.argtypes = [i32, i32]
        L.ti_gemm_packed_rows_for.argtypes = [i32, i32, i32, i32]
        L.ti_gemm_tile_plan.argtypes = [i32, i32, i32, i32, C.c_int64, vp, vp, vp]
        L.ti_rmsnorm_f16.argtypes = [vp, i32, vp, f32, vp, i32, i32, i32, vp]
        L.ti_rmsnorm_f16_packed.argtypes = [vp, i32, vp, f32, vp, i32, i32, vp]
        L.ti_attn_workspace_bytes.argtypes = [i32, i32, i32, i32]
        L.ti_attn_workspace_bytes.restype = sz
        L.ti_attn_decode.argtypes = [vp, vp, vp, i64, i32, vp, i32, i32, i32, i32, i32, vp, vp, vp]
        L.ti_attn_decode_packed.argtypes = [vp, vp, vp, i64, i32, vp, i32, i32, i32, i32, i32, vp, vp, vp]
        L.ti_attn_prefill.argtypes = [vp, vp, vp, i32, vp, i32, i32, i32, i32, vp, vp]
        L.ti_attn_prefill_set_kernel.argtypes = [i32]
        if hasattr(L, "ti_sample_device"):
            L.ti_sample_device.argtypes = [vp, i32, i32, i32, f32, i32, f32, vp, vp, vp, vp]
        if hasattr(L, "ti_sample_device_ws"):
            L.ti_sample_device_ws.argtypes = [vp, i32, i32, i32, f32, i32, f32, vp, vp, vp, vp, vp]
            L.ti_sample_workspace_bytes.argtypes = [i32, i32]
            L.ti_sample_workspace_bytes.restype = sz
            L.ti_engine_generate_sampled.argtypes = [vp, i32, vp, vp, i32, vp, i32, f32, i32, f32, vp, vp, vp]
        if hasattr(L, "ti_engine_serve"):
            L.ti_engine_serve.argtypes = [vp, i32, vp, vp, i32, i32, i32, vp, vp]
        if hasattr(L, "ti_engine_beam_search"):
            L.ti_engine_beam_search.argtypes = [vp, vp, i32, i32, i32, f32, i32, f32, f32, i32, vp, vp, vp, vp,
                                                C.POINTER(C.c_int)]
        if hasattr(L, "ti_attn_decode_partials"):
            L.ti_attn_decode_partials.argtypes = [vp, vp, vp, i64, i32, vp, i32, i32, i32, i32, i32, vp, vp, vp]
        L.ti_step_begin.argtypes = [C.POINTER(StepArgs), vp]
        L.ti_matmul_f32.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, vp]
        L.ti_rms_norm_f32.argtypes = [vp, vp, vp, i32, i32, f32, vp]
        L.ti_rope_f32.argtypes = [vp, vp, vp, i32, i32, i32, i32, i32, vp]
        for n in ("ti_silu_f32", "ti_relu_f32"):
            getattr(L, n).argtypes = [vp, vp, i64, vp]
        for n in ("ti_add_f32", "ti_mul_f32"):
            getattr(L, n).argtypes = [vp, vp, vp, i64, vp]
        L.ti_softmax_f32.argtypes = [vp, vp, i32, i32, f32, vp]
        L.ti_attention_f32.argtypes = [vp, vp, vp, vp, vp, i32, i32, i32, i32, vp]
        L.ti_argmax_f32.argtypes = [vp, vp, i32, i32, vp]
        L.ti_engine_create.argtypes = [C.POINTER(EngineConfig), C.POINTER(vp)]
        L.ti_engine_destroy.argtypes = [vp]
        L.ti_engine_get_stream.argtypes = [vp, C.POINTER(vp)]
        L.ti_engine_memory.argtypes = [vp, C.POINTER(sz), C.POINTER(sz)]
        L.ti_engine_set_tensor.argtypes = [vp, i32, i32, vp, i32]
        if hasattr(L, "ti_engine_set_tensor_q"):
            L.ti_engine_set_tensor_q.argtypes = [vp, i32, i32, vp, vp]
            L.ti_wpack_q_host.argtypes = [vp, vp, i32, i32, i32, i32, i32, i32, vp, vp]
        if hasattr(L, "ti_engine_set_tensor_q1"):
            L.ti_engine_set_tensor_q1.argtypes = [vp, i32, i32, vp, vp, vp]
            L.ti_wpack_q1_host.argtypes = [vp, vp, vp, i32, i32, i32, i32, i32, vp, vp]
        L.ti_engine_synth.argtypes = [vp, u64, f32]
        L.ti_engine_fill_kv.argtypes = [vp, i32, i32, u64]
        L.ti_engine_generate.argtypes = [vp, i32, vp, vp, i32, vp, i32, vp, vp]
        L.ti_engine_step.argtypes = [vp, i32, vp, vp, vp]
        L.ti_engine_set_prefill.argtypes = [vp, i32]
        if hasattr(L, "ti_engine_set_stop"):
            L.ti_engine_set_stop.argtypes = [vp, C.c_int32]
            L.ti_engine_counters.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        if hasattr(L, "ti_engine_set_fold"):   # (older TI_LIB builds in A/B runs lack it)
            L.ti_gemm_grid.argtypes = [i32, i32, i32]
            L.ti_engine_set_fold.argtypes = [vp, i32, C.POINTER(C.c_int)]
        if hasattr(L, "ti_qkv_attn_partials"):   # (older TI_LIB builds in A/B runs lack it)
            L.ti_engine_set_qkv_attn.argtypes = [vp, i32, C.POINTER(C.c_int)]
            L.ti_qkv_attn_partials.argtypes = [vp, vp, i32, vp, vp, i32, f32, vp, vp, vp, vp, i32, i32, i32, i32,
                                               i32, i32, vp, vp, vp, vp]
            L.ti_qkv_attn_xchg_bytes.argtypes = [i32, i32]
            L.ti_qkv_attn_supported.argtypes = [i32, i32, i32, i32, i32, i32]
            L.ti_qkv_attn_xchg_bytes.restype = sz
            L.ti_qkv_attn_error_offset.argtypes = [i32, i32]
            L.ti_qkv_attn_error_offset.restype = sz
            L.ti_qkv_attn_part_o_elems.argtypes = [i32, i32, i32]
            L.ti_qkv_attn_part_o_elems.restype = sz
            L.ti_qkv_attn_part_ml_elems.argtypes = [i32, i32, i32]
            L.ti_qkv_attn_part_ml_elems.restype = sz
        L.ti_engine_compat_step.argtypes = [vp, i32, vp]
        L.ti_engine_replay_prepare.argtypes = [vp, i32, i32, i32]
        L.ti_engine_replay_run.argtypes = [vp, i32]
        L.ti_engine_sync.argtypes = [vp]
        L.ti_engine_last_tokens.argtypes = [vp, i32, vp]
        L.ti_engine_time_kernel.argtypes = [vp, i32, i32, i32, i32, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        if hasattr(L, "ti_engine_stamp_steps"):   # (older TI_LIB builds in A/B runs lack it)
            L.ti_engine_stamp_steps.argtypes = [vp, i32, i32, vp, vp, C.POINTER(C.c_int)]
        L.ti_hbm_calibrate.argtypes = [sz, i32, C.POINTER(C.c_double), C.POINTER(C.c_double), vp]
        L.ti_gemm_kernel_name.argtypes = [i32, i32, i32, i32, i32, C.c_char_p, i32]
        L.ti_rope_table.argtypes = [vp, i32, i32, f32, vp]
        L.ti_sample_token.argtypes = [vp, i32, f32, i32, f32, f32, C.POINTER(C.c_int), C.POINTER(C.c_float)]
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != TI_OK:
        raise TiError(f"ti error {rc}: {lib().ti_last_error().decode()}")


def device_count() -> int:
    n = C.c_int(0)
    check(lib().ti_device_count(C.byref(n)))
    return n.value


def init(device: int = 0) -> None:
    check(lib().ti_init(device))


def _ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


class DeviceBuffer:
    """Owning device allocation (ti_malloc / ti_free)."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(lib().ti_malloc(C.byref(p), max(int(nbytes), 16)))
        self.ptr = p.value
        self.nbytes = int(nbytes)

    @classmethod
    def from_array(cls, a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        b.upload(a)
        return b

    def upload(self, a: np.ndarray) -> None:
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        check(lib().ti_memcpy_h2d(self.ptr, _ptr(a), a.nbytes, None))

    def download(self, dtype, shape) -> np.ndarray:
        out = np.empty(shape, dtype=dtype)
        assert out.nbytes <= self.nbytes
        check(lib().ti_memcpy_d2h(_ptr(out), self.ptr, out.nbytes, None))
        return out

    def zero(self) -> None:
        check(lib().ti_memset(self.ptr, 0, self.nbytes, None))

    def free(self) -> None:
        if getattr(self, "ptr", None):
            lib().ti_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def hbm_calibrate(nbytes: int = 1 << 30, reps: int = 5) -> tuple[float, float]:
    """(read GB/s, device-copy GB/s) of this GPU now: the same-run calibration of bench lines."""
    r, c = C.c_double(), C.c_double()
    check(lib().ti_hbm_calibrate(nbytes, reps, C.byref(r), C.byref(c), None))
    return r.value, c.value


def gemm_kernel_name(bits: int, x_kind: int, M: int, N: int, K: int) -> str:
    buf = C.create_string_buffer(64)
    check(lib().ti_gemm_kernel_name(bits, x_kind, M, N, K, buf, 64))
    return buf.value.decode()


def sync() -> None:
    check(lib().ti_device_sync())


# ------------------------------------------------------------------ packing helpers
def wpack_host(w: np.ndarray, bits: int, n_total: int | None = None, scale_mode: int = SCALE_GROUP,
               row_map: int = ROWS_CONCAT, row_offset: int = 0, tiles=None, scales=None):
    """Quantize + pack a reference-layout [K][N] fp32 weight into (tiles bytes, fp16 scale bits)."""
    w = np.ascontiguousarray(w, np.float32)
    K, N = w.shape
    n_total = n_total or N
    L = lib()
    if tiles is None:
        tiles = np.zeros(L.ti_wpack_tile_bytes(bits, K, n_total), np.uint8)
    if scales is None:
        scales = np.zeros(max(L.ti_wpack_scale_bytes(bits, K, n_total) // 2, 1), np.uint16)
    check(L.ti_wpack_host(_ptr(w), K, N, n_total, bits, scale_mode, row_map, row_offset, _ptr(tiles),
                          _ptr(scales) if bits != 16 else None))
    return tiles, scales


def packed_index(m, k, K):
    """TI_PACKED_INDEX (include/ti_hip.h): element (m, k) of a TI_X_F16_PACKED operand (numpy arrays ok)."""
    kt = K // 128
    return (((((m >> 4) * kt + (k >> 7)) * 4 + ((k >> 3) & 3)) * 64 + ((k >> 5) & 3) * 16 + (m & 15)) * 8 + (k & 7))


def pack_rows(x):
    """Row-major [M][K] -> TI_X_F16_PACKED order (rows padded to a multiple of 16)."""
    M, K = x.shape
    Mp = (M + 15) // 16 * 16
    out = np.zeros(Mp * K, x.dtype)
    mm, kk = np.meshgrid(np.arange(M), np.arange(K), indexing="ij")
    out[packed_index(mm, kk, K)] = x
    return out


def unpack_rows(p, M, K):
    mm, kk = np.meshgrid(np.arange(M), np.arange(K), indexing="ij")
    return p[packed_index(mm, kk, K)]


def rope_table(pos, head_dim: int, theta: float) -> np.ndarray:
    """(cos, sin) table [len(pos)][head_dim/2][2] from the product's host code (ti_rope_table,
    the reference formula in fp32 libm)."""
    p = np.ascontiguousarray(pos, np.float32).reshape(-1)
    out = np.zeros((p.size, head_dim // 2, 2), np.float32)
    check(lib().ti_rope_table(_ptr(p), p.size, head_dim, theta, _ptr(out)))
    return out


def sample_token(logits, temperature=1.0, top_k=1, top_p=0.9, u=0.5):
    """The product's host sampler (ti_sample_token) -> (token, logprob)."""
    lg = np.ascontiguousarray(logits, np.float32).reshape(-1)
    t, lp = C.c_int(), C.c_float()
    check(lib().ti_sample_token(_ptr(lg), lg.size, temperature, top_k, top_p, u, C.byref(t), C.byref(lp)))
    return t.value, lp.value


class Engine:
    """ctypes wrapper over ti_engine (include/ti_engine.h)."""

    def __init__(self, vocab, hidden, layers, heads, kv_heads, head_dim, inter, bits=4, max_seq=2048,
                 max_batch=1, rope_theta=10000.0, eps=1e-5, compat=False, device=0, attn_splits=0):
        self.cfg = EngineConfig(vocab, hidden, layers, heads, kv_heads, head_dim, inter, rope_theta, eps, bits,
                                max_seq, max_batch, int(compat), device, attn_splits)
        h = C.c_void_p()
        check(lib().ti_engine_create(C.byref(self.cfg), C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().ti_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_tensor_q(self, slot, layer, q, d):
        """Exact group-32 weight (engine bits 4/8 | BITS_G32): q int8 [K][N], d fp16 [K/32][N]."""
        qa = np.ascontiguousarray(q, np.int8)
        da = np.ascontiguousarray(d, np.float16).view(np.uint16)
        check(lib().ti_engine_set_tensor_q(self.h, slot, layer, qa.ctypes.data, da.ctypes.data))


    def set_tensor_q1(self, slot, layer, q, d, m):
        """Exact GGUF Q4_1 blocks (engine bits 4 | BITS_G32 | BITS_AFF): q uint8 [K][N] (0..15),
        d, m fp16 [K/32][N]; weight = d * q + m."""
        qa = np.ascontiguousarray(q, np.uint8)
        da = np.ascontiguousarray(d, np.float16).view(np.uint16)
        ma = np.ascontiguousarray(m, np.float16).view(np.uint16)
        check(lib().ti_engine_set_tensor_q1(self.h, slot, layer, qa.ctypes.data, da.ctypes.data, ma.ctypes.data))
    def set_tensor(self, slot, layer, data, scale_mode=SCALE_GROUP):
        a = np.ascontiguousarray(data, np.float32)
        check(lib().ti_engine_set_tensor(self.h, slot, layer, _ptr(a), scale_mode))

    def synth(self, seed, norm_jitter=0.0):
        check(lib().ti_engine_synth(self.h, seed, norm_jitter))

    def fill_kv(self, stream, n, seed):
        check(lib().ti_engine_fill_kv(self.h, stream, n, seed))

    def generate(self, prompts, max_new, start_pos=None, want_logits=False):
        n = len(prompts)
        stride = max(len(p) for p in prompts)
        P = np.zeros((n, stride), np.int32)
        for i, p in enumerate(prompts):
            P[i, : len(p)] = p
        lens = np.array([len(p) for p in prompts], np.int32)
        out = np.zeros((n, max_new), np.int32)
        sp = None if start_pos is None else np.ascontiguousarray(start_pos, np.int32)
        logits = np.zeros((n, self.cfg.vocab), np.float32) if want_logits else None
        check(lib().ti_engine_generate(self.h, n, _ptr(P), _ptr(lens), stride, None if sp is None else _ptr(sp),
                                       max_new, _ptr(out), None if logits is None else _ptr(logits)))
        return (out, logits) if want_logits else out

    def generate_sampled(self, prompts, max_new, temperature, top_k, top_p, draws, start_pos=None):
        """ti_engine_generate_sampled: tokens [n][max_new] and log-probs [n][max_new]."""
        n = len(prompts)
        stride = max(len(p) for p in prompts)
        P = np.zeros((n, stride), np.int32)
        for i, p in enumerate(prompts):
            P[i, : len(p)] = p
        lens = np.array([len(p) for p in prompts], np.int32)
        d = np.ascontiguousarray(draws, np.float32).reshape(n, max_new)
        out = np.zeros((n, max_new), np.int32)
        lp = np.zeros((n, max_new), np.float32)
        sp = None if start_pos is None else np.ascontiguousarray(start_pos, np.int32)
        check(lib().ti_engine_generate_sampled(self.h, n, _ptr(P), _ptr(lens), stride, None if sp is None else _ptr(sp),
                                               max_new, temperature, top_k, top_p, _ptr(d), _ptr(out), _ptr(lp)))
        return out, lp

    def beam_search(self, prompt, max_new, beam_size, temperature=1.0, top_k=0, top_p=1.0, length_penalty=1.0,
                    eos=2):
        """ti_engine_beam_search -> [(new tokens, log_prob, normalised score, finished)], best first."""
        p = np.ascontiguousarray(prompt, np.int32)
        out = np.zeros((beam_size, max_new), np.int32)
        lp, sc = np.zeros(beam_size, np.float32), np.zeros(beam_size, np.float32)
        fin, cnt = np.zeros(beam_size, np.int32), C.c_int(0)
        check(lib().ti_engine_beam_search(self.h, _ptr(p), p.size, max_new, beam_size, temperature, top_k, top_p,
                                          length_penalty, eos, _ptr(out), _ptr(lp), _ptr(sc), _ptr(fin),
                                          C.byref(cnt)))
        return [([int(t) for t in out[r] if t >= 0], float(lp[r]), float(sc[r]), bool(fin[r]))
                for r in range(cnt.value)]

    def serve(self, prompts, max_new, eos=2, chunk=16):
        """ti_engine_serve (continuous batching): each request's new tokens, in request order."""
        flat = np.ascontiguousarray([t for p in prompts for t in p], np.int32)
        offs = np.ascontiguousarray(np.cumsum([0] + [len(p) for p in prompts]), np.int32)
        out = np.zeros((len(prompts), max_new), np.int32)
        n = np.zeros(len(prompts), np.int32)
        check(lib().ti_engine_serve(self.h, len(prompts), _ptr(flat), _ptr(offs), max_new, eos, chunk, _ptr(out),
                                    _ptr(n)))
        return [out[r, : n[r]].tolist() for r in range(len(prompts))]

    def set_prefill(self, rows):
        """Prompt tokens per prefill chunk (0 = consume prompts one token per decode step)."""
        check(lib().ti_engine_set_prefill(self.h, rows))

    def set_stop(self, token=-1):
        """Stop token of generate / generate_sampled (-1: none): the device loop ends in chunks once
        every stream has emitted it (ti_engine_set_stop)."""
        check(lib().ti_engine_set_stop(self.h, token))

    def counters(self):
        """(decode step-graph replays, prefill chunks) run by this engine (ti_engine_counters)."""
        a, b = C.c_uint64(0), C.c_uint64(0)
        check(lib().ti_engine_counters(self.h, C.byref(a), C.byref(b)))
        return int(a.value), int(b.value)

    def set_fold(self, on=None) -> bool:
        """Folded rms_norm hand-off on/off (None: query); returns whether 1-stream steps use it."""
        act = C.c_int(0)
        check(lib().ti_engine_set_fold(self.h, -1 if on is None else int(bool(on)), C.byref(act)))
        return bool(act.value)

    def set_qkv_attn(self, on=None) -> bool:
        """QKV + attention in one launch on/off (None: query); returns whether 1-stream steps use it."""
        act = C.c_int(0)
        check(lib().ti_engine_set_qkv_attn(self.h, -1 if on is None else int(bool(on)), C.byref(act)))
        return bool(act.value)

    def step(self, tokens, pos):
        t = np.ascontiguousarray(tokens, np.int32)
        p = np.ascontiguousarray(pos, np.int32)
        logits = np.zeros((t.size, self.cfg.vocab), np.float32)
        check(lib().ti_engine_step(self.h, t.size, _ptr(t), _ptr(p), _ptr(logits)))
        return logits

    def compat_step(self, offset):
        logits = np.zeros(self.cfg.vocab, np.float32)
        check(lib().ti_engine_compat_step(self.h, offset, _ptr(logits)))
        return logits

    def replay_prepare(self, n_streams, kv_len, start_token):
        check(lib().ti_engine_replay_prepare(self.h, n_streams, kv_len, start_token))

    def replay_run(self, steps):
        check(lib().ti_engine_replay_run(self.h, steps))

    def sync(self):
        check(lib().ti_engine_sync(self.h))

    def last_tokens(self, n):
        t = np.zeros(n, np.int32)
        check(lib().ti_engine_last_tokens(self.h, n, _ptr(t)))
        return t

    def time_kernel(self, which, n_streams, kv_len, reps):
        us, by = C.c_double(), C.c_double()
        check(lib().ti_engine_time_kernel(self.h, which, n_streams, kv_len, reps, C.byref(us), C.byref(by)))
        return us.value, by.value

    STAMP_FIELDS = ("span_us", "period_us", "entry_skew_us", "wave_skew_us", "tail_us", "gap_us", "cu_shared_wgs",
                    "ph1_us", "ph2_us", "ph3_us", "ph4_us", "ph5_us", "ph6_us", "stream_skew_us")
    STAMP_TAGS = ("begin", "qkv", "attention", "o", "gate_up", "down", "lm_head", "other")
    STAMP_KINDS = ("other", "gemv", "attn", "step_begin", "rows", "tile", "rmsnorm", "mb")

    def stamp_steps(self, steps=20, cap=4096):
        """In-step launch timing of the replay step (ti_engine_stamp_steps): one dict per launch with
        kind, tag, workgroups and the per-launch means of STAMP_FIELDS in us."""
        info = np.zeros((cap, 3), np.int32)
        t = np.zeros((cap, len(self.STAMP_FIELDS)), np.float64)
        n = C.c_int(0)
        check(lib().ti_engine_stamp_steps(self.h, steps, cap, _ptr(info), _ptr(t), C.byref(n)))
        out = []
        for i in range(min(n.value, cap)):
            d = {"kind": self.STAMP_KINDS[info[i, 0]], "tag": self.STAMP_TAGS[info[i, 1]], "workgroups": int(info[i, 2])}
            d.update({k: float(t[i, j]) for j, k in enumerate(self.STAMP_FIELDS)})
            out.append(d)
        return out

    def memory(self):
        w, k = C.c_size_t(), C.c_size_t()
        check(lib().ti_engine_memory(self.h, C.byref(w), C.byref(k)))
        return w.value, k.value
