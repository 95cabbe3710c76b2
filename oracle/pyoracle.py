"""TEST INFRASTRUCTURE ONLY -- ctypes bindings for the CPU oracle and the compiled reference.

`Oracle` wraps oracle/_build/libti_oracle.so (the plain-C restatement in ti_oracle.c);
`Reference` wraps oracle/_ref/libti_ref.so (the unmodified reference sources + ref_shim.cpp).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "_build", "libti_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libti_ref.so")

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i8p = np.ctypeslib.ndpointer(np.int8, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
SZ = C.c_size_t
_FWD = C.CFUNCTYPE(C.c_size_t, C.c_void_p, C.POINTER(C.c_int32), C.c_size_t, C.POINTER(C.POINTER(C.c_float)))


def build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


class ModelConfig(C.Structure):
    _fields_ = [("vocab", C.c_int), ("hidden", C.c_int), ("layers", C.c_int), ("heads", C.c_int),
                ("kv_heads", C.c_int), ("head_dim", C.c_int), ("inter", C.c_int),
                ("rope_theta", C.c_float), ("eps", C.c_float), ("bits", C.c_int),
                ("group", C.c_int), ("max_seq", C.c_int)]


_FP = C.POINTER(C.c_float)
_FPP = C.POINTER(_FP)


class _OrModel(C.Structure):
    """Mirror of or_model (ti_oracle.h) -- read-only access to the materialised weights."""
    _fields_ = [("cfg", ModelConfig), ("emb", _FP), ("attn_norm", _FPP), ("ffn_norm", _FPP), ("wq", _FPP),
                ("wk", _FPP), ("wv", _FPP), ("wo", _FPP), ("wg", _FPP), ("wu", _FPP), ("wd", _FPP),
                ("out_norm", _FP), ("lm_head", _FP), ("kc", _FPP), ("vc", _FPP), ("len", C.c_int)]


class Oracle:
    """The plain-C restatement (ti_oracle.c)."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build_oracle()
        L = self.lib = C.CDLL(path)
        L.or_matmul.argtypes = [_f32p, _f32p, _f32p, SZ, SZ, SZ]
        L.or_rms_norm.argtypes = [_f32p, _f32p, _f32p, SZ, SZ, C.c_float]
        L.or_apply_rope.argtypes = [_f32p, _f32p, SZ, SZ, SZ, SZ, _f32p, C.c_int, C.c_float]
        for n in ("or_silu", "or_relu"):
            getattr(L, n).argtypes = [_f32p, _f32p, SZ]
        for n in ("or_add", "or_multiply"):
            getattr(L, n).argtypes = [_f32p, _f32p, _f32p, SZ]
        L.or_softmax.argtypes = [_f32p, _f32p, SZ, SZ, C.c_float]
        L.or_attention_incremental.argtypes = [_f32p, _f32p, _f32p, _f32p, SZ, SZ, SZ]
        L.or_multi_head_attention.argtypes = [_f32p, _f32p, _f32p, _f32p, SZ, SZ, SZ, SZ]
        L.or_quant_info.argtypes = [_f32p, SZ, C.c_int, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.or_quantize_int8.argtypes = [_f32p, _i8p, SZ, C.c_float, C.c_float]
        L.or_quantize_int4.argtypes = [_f32p, _i32p, SZ, C.c_float, C.c_float]
        L.or_dequantize_int8.argtypes = [_i8p, _f32p, SZ, C.c_float, C.c_float]
        L.or_dequantize_int4.argtypes = [_i32p, _f32p, SZ, C.c_float, C.c_float]
        L.or_quantize_groups.argtypes = [_f32p, SZ, SZ, C.c_int, C.c_int, C.c_int, _i8p, _u16p]
        L.or_dequantize_groups.argtypes = [_i8p, _u16p, SZ, SZ, C.c_int, _f32p]
        L.or_synth_linear.argtypes = [C.c_uint64, C.c_uint32, SZ, SZ, _f32p]
        L.or_synth_unit.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64]
        L.or_synth_unit.restype = C.c_float
        L.or_model_synth.argtypes = [C.POINTER(ModelConfig), C.c_uint64, C.c_float]
        L.or_model_synth.restype = C.c_void_p
        L.or_model_free.argtypes = [C.c_void_p]
        L.or_model_fill_kv.argtypes = [C.c_void_p, C.c_int, C.c_uint64]
        L.or_decode_step.argtypes = [C.c_void_p, C.c_int, _f32p, C.c_int]
        L.or_decode_step.restype = C.c_int
        L.or_plumbing_generate.argtypes = [SZ, SZ, SZ, _i32p, SZ, SZ, SZ, _i32p, _f32p]
        L.or_plumbing_generate.restype = SZ
        L.or_sample_token.argtypes = [_f32p, SZ, C.c_float, SZ, C.c_float, C.c_float, C.POINTER(C.c_float)]
        L.or_sample_token.restype = C.c_int
        L.or_sample_probs.argtypes = [_f32p, SZ, C.c_float, SZ, C.c_float, _f32p]
        L.or_sample_probs.restype = None
        L.or_beam_search.argtypes = [_FWD, C.c_void_p, _i32p, SZ, SZ, SZ, C.c_float, SZ, C.c_float, C.c_float,
                                     C.c_int, _i32p, _i32p, _f32p, _f32p, _i32p, C.POINTER(C.c_float)]
        L.or_beam_search.restype = C.c_int
        L.or_plumbing_forward_rows.argtypes = [SZ, SZ, SZ, SZ, _f32p]
        L.or_plumbing_forward_rows.restype = None
        L.or_qmodel_synth.argtypes = [C.POINTER(ModelConfig), C.c_uint64, C.c_float]
        L.or_qmodel_synth.restype = C.c_void_p
        L.or_qmodel_free.argtypes = [C.c_void_p]
        L.or_qmodel_fill_kv.argtypes = [C.c_void_p, C.c_int, C.c_uint64]
        L.or_qmodel_set_len.argtypes = [C.c_void_p, C.c_int]
        L.or_qmodel_set_len.restype = C.c_int
        L.or_qmodel_step.argtypes = [C.c_void_p, C.c_int, _f32p]
        L.or_qmodel_step.restype = C.c_int
        L.or_half_to_float.argtypes = [C.c_uint16]
        L.or_half_to_float.restype = C.c_float
        L.or_float_to_half.argtypes = [C.c_float]
        L.or_float_to_half.restype = C.c_uint16

    # ---- ops
    def matmul(self, a, b):
        a, b = f32(a), f32(b)
        K, N = b.shape
        rows = a.size // K
        y = np.empty(rows * N, np.float32)
        self.lib.or_matmul(a.reshape(-1), b.reshape(-1), y, rows, K, N)
        return y.reshape(a.shape[:-1] + (N,))

    def rms_norm(self, x, w, eps=1e-5):
        x, w = f32(x), f32(w)
        y = np.empty_like(x)
        n = x.shape[-1]
        self.lib.or_rms_norm(x.reshape(-1), w, y.reshape(-1), x.size // n, n, eps)
        return y

    def apply_rope(self, x, pos, theta=10000.0):
        """x: [B,heads,S,D] (4-D) or [B,S,D] (3-D); pos: [S] or [B,S]."""
        x, pos = f32(x), f32(pos)
        if x.ndim == 3:
            B, S, D = x.shape
            heads = 1
        else:
            B, heads, S, D = x.shape
        y = np.empty_like(x)
        self.lib.or_apply_rope(x.reshape(-1), y.reshape(-1), B, heads, S, D, pos.reshape(-1),
                               1 if pos.ndim == 2 else 0, theta)
        return y

    def _unary(self, name, x):
        x = f32(x)
        y = np.empty_like(x)
        getattr(self.lib, name)(x.reshape(-1), y.reshape(-1), x.size)
        return y

    def silu(self, x):
        return self._unary("or_silu", x)

    def relu(self, x):
        return self._unary("or_relu", x)

    def add(self, a, b):
        a, b = f32(a), f32(b)
        y = np.empty_like(a)
        self.lib.or_add(a.reshape(-1), b.reshape(-1), y.reshape(-1), a.size)
        return y

    def multiply(self, a, b):
        a, b = f32(a), f32(b)
        y = np.empty_like(a)
        self.lib.or_multiply(a.reshape(-1), b.reshape(-1), y.reshape(-1), a.size)
        return y

    def softmax(self, x, temperature=1.0):
        x = f32(x)
        n = x.shape[-1]
        y = np.empty_like(x)
        self.lib.or_softmax(x.reshape(-1), y.reshape(-1), x.size // n, n, temperature)
        return y

    def attention_incremental(self, q, k, v):
        q, k, v = f32(q), f32(k), f32(v)
        B, S, D = k.shape
        y = np.empty((B, 1, D), np.float32)
        self.lib.or_attention_incremental(q.reshape(-1), k.reshape(-1), v.reshape(-1), y.reshape(-1), B, S, D)
        return y

    def multi_head_attention(self, q, k, v, heads):
        q, k, v = f32(q), f32(k), f32(v)
        B, S, H = k.shape
        y = np.empty((B, 1, H), np.float32)
        self.lib.or_multi_head_attention(q.reshape(-1), k.reshape(-1), v.reshape(-1), y.reshape(-1), B, S, H, heads)
        return y

    def quant_info(self, x, bits, symmetric=True):
        x = f32(x).reshape(-1)
        s, z = C.c_float(), C.c_float()
        self.lib.or_quant_info(x, x.size, bits, int(symmetric), C.byref(s), C.byref(z))
        return s.value, z.value

    def quantize(self, x, bits, scale, zp):
        x = f32(x).reshape(-1)
        if bits == 8:
            q = np.empty(x.size, np.int8)
            self.lib.or_quantize_int8(x, q, x.size, scale, zp)
            return q.astype(np.int32)
        q = np.empty(x.size, np.int32)
        self.lib.or_quantize_int4(x, q, x.size, scale, zp)
        return q

    def dequantize(self, q, bits, scale, zp):
        y = np.empty(q.size, np.float32)
        if bits == 8:
            self.lib.or_dequantize_int8(np.ascontiguousarray(q, np.int8).reshape(-1), y, q.size, scale, zp)
        else:
            self.lib.or_dequantize_int4(np.ascontiguousarray(q, np.int32).reshape(-1), y, q.size, scale, zp)
        return y

    def quantize_groups(self, w, bits, group=128, scale_mode=0):
        """w [K][N] -> (q [N][K] int8, scales [N][K/group] fp16 bits)."""
        w = f32(w)
        K, N = w.shape
        q = np.empty((N, K), np.int8)
        s = np.empty((N, K // group), np.uint16)
        self.lib.or_quantize_groups(w.reshape(-1), K, N, bits, group, scale_mode, q.reshape(-1), s.reshape(-1))
        return q, s

    def dequantize_groups(self, q, s, group=128):
        N, K = q.shape
        w = np.empty((K, N), np.float32)
        self.lib.or_dequantize_groups(np.ascontiguousarray(q).reshape(-1), np.ascontiguousarray(s).reshape(-1),
                                      K, N, group, w.reshape(-1))
        return w

    def synth_linear(self, seed, tid, K, N):
        w = np.empty((K, N), np.float32)
        self.lib.or_synth_linear(seed, tid, K, N, w.reshape(-1))
        return w

    def sample_token(self, logits, temperature=1.0, top_k=1, top_p=0.9, u=0.5):
        lg = f32(logits).reshape(-1)
        lp = C.c_float()
        t = self.lib.or_sample_token(lg, lg.size, temperature, top_k, top_p, u, C.byref(lp))
        return t, lp.value

    def sample_probs(self, logits, temperature=1.0, top_k=1, top_p=0.9):
        lg = f32(logits).reshape(-1)
        pr = np.empty(lg.size, np.float32)
        self.lib.or_sample_probs(lg, lg.size, temperature, top_k, top_p, pr)
        return pr

    def beam_search(self, forward, prompt, max_new, beam, temperature=1.0, top_k=0, top_p=1.0,
                    length_penalty=1.0, eos=2):
        """or_beam_search (beam_search_decode restated) over forward(tokens) -> logits:
        ([(new tokens, log_prob, normalised score, finished)] best first, smallest decision gap)."""
        keep = {}

        def cb(_ctx, toks, n, out):
            lg = np.ascontiguousarray(forward([toks[i] for i in range(n)]), np.float32)
            keep["lg"] = lg
            out[0] = lg.ctypes.data_as(C.POINTER(C.c_float))
            return lg.size

        fn = _FWD(cb)
        p = np.ascontiguousarray(prompt, np.int32)
        toks = np.zeros(beam * max(max_new, 1), np.int32)
        nt, fin = np.zeros(beam, np.int32), np.zeros(beam, np.int32)
        lp, sc, gap = np.zeros(beam, np.float32), np.zeros(beam, np.float32), C.c_float()
        n = self.lib.or_beam_search(fn, None, p, p.size, max_new, beam, temperature, top_k, top_p, length_penalty,
                                    eos, toks, nt, lp, sc, fin, C.byref(gap))
        if n < 0:
            raise RuntimeError(f"or_beam_search: {n}")
        m = max(max_new, 1)
        return ([(toks[r * m: r * m + nt[r]].tolist(), float(lp[r]), float(sc[r]), bool(fin[r])) for r in range(n)],
                gap.value)

    def plumbing_forward_rows(self, vocab, hidden, layers, n):
        out = np.empty(n * vocab, np.float32)
        self.lib.or_plumbing_forward_rows(vocab, hidden, layers, n, out)
        return out

    def plumbing_generate(self, vocab, hidden, layers, prompt, max_new, max_seq=2048):
        p = np.ascontiguousarray(prompt, np.int32)
        out = np.zeros(len(prompt) + max_new, np.int32)
        logits = np.zeros(vocab, np.float32)
        n = self.lib.or_plumbing_generate(vocab, hidden, layers, p, p.size, max_new, max_seq, out, logits)
        return out[:n].tolist(), logits


class OracleModel:
    """A synthetic Llama-shape model materialised in the oracle (dequantized fp32)."""

    def __init__(self, oracle: Oracle, cfg: dict, seed: int, norm_jitter: float = 0.0):
        self.o = oracle
        self.cfg = cfg
        c = ModelConfig(**cfg)
        self.ptr = oracle.lib.or_model_synth(C.byref(c), seed, norm_jitter)

    def fill_kv(self, n, seed):
        self.o.lib.or_model_fill_kv(self.ptr, n, seed)

    def weights(self):
        """The model's fp32 tensors under the reference's weight names
        (inference_engine.cpp:483-563 "layers.N.attention.*" / "feed_forward.w1|w2|w3"),
        [K][N] layout, copied out of the oracle."""
        m = C.cast(self.ptr, C.POINTER(_OrModel)).contents
        c = self.cfg
        H, I, V = c["hidden"], c["inter"], c["vocab"]
        qd, kvd = c["heads"] * c["head_dim"], c["kv_heads"] * c["head_dim"]

        def arr(p, *shape):
            return np.ctypeslib.as_array(p, shape=(int(np.prod(shape)),)).reshape(shape).copy()

        out = {"token_embeddings.weight": arr(m.emb, V, H), "norm.weight": arr(m.out_norm, H),
               "lm_head.weight": arr(m.lm_head, H, V)}
        for l in range(c["layers"]):
            p = f"layers.{l}."
            out[p + "attention.q_proj.weight"] = arr(m.wq[l], H, qd)
            out[p + "attention.k_proj.weight"] = arr(m.wk[l], H, kvd)
            out[p + "attention.v_proj.weight"] = arr(m.wv[l], H, kvd)
            out[p + "attention.o_proj.weight"] = arr(m.wo[l], qd, H)
            out[p + "feed_forward.w3.weight"] = arr(m.wg[l], H, I)     # gate
            out[p + "feed_forward.w1.weight"] = arr(m.wu[l], H, I)     # up
            out[p + "feed_forward.w2.weight"] = arr(m.wd[l], I, H)     # down
            out[p + "attention_norm.weight"] = arr(m.attn_norm[l], H)
            out[p + "ffn_norm.weight"] = arr(m.ffn_norm[l], H)
        return out

    def set_weights(self, w):
        """Overwrite the oracle's tensors in place from a dict shaped like weights() (e.g. the
        same tensors after a GGUF quantize -> dequantize round trip)."""
        m = C.cast(self.ptr, C.POINTER(_OrModel)).contents
        c = self.cfg
        ptrs = {"token_embeddings.weight": m.emb, "norm.weight": m.out_norm, "lm_head.weight": m.lm_head}
        for l in range(c["layers"]):
            p = f"layers.{l}."
            ptrs.update({p + "attention.q_proj.weight": m.wq[l], p + "attention.k_proj.weight": m.wk[l],
                         p + "attention.v_proj.weight": m.wv[l], p + "attention.o_proj.weight": m.wo[l],
                         p + "feed_forward.w3.weight": m.wg[l], p + "feed_forward.w1.weight": m.wu[l],
                         p + "feed_forward.w2.weight": m.wd[l], p + "attention_norm.weight": m.attn_norm[l],
                         p + "ffn_norm.weight": m.ffn_norm[l]})
        for k, v in w.items():
            a = np.ascontiguousarray(v, np.float32).reshape(-1)
            np.ctypeslib.as_array(ptrs[k], shape=(a.size,))[:] = a

    def step(self, token, kv_round_f16=True):
        logits = np.empty(self.cfg["vocab"], np.float32)
        t = self.o.lib.or_decode_step(self.ptr, int(token), logits, int(kv_round_f16))
        return t, logits

    def close(self):
        if self.ptr:
            self.o.lib.or_model_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.close()


class OracleDeepModel:
    """The same synthetic model at full depth (ti_oracle_deep.c): weights kept as group-quantized
    int8 + scales, steps bit-identical to OracleModel.step(kv_round_f16=True), multi-threaded."""

    def __init__(self, oracle: Oracle, cfg: dict, seed: int, norm_jitter: float = 0.0):
        self.o = oracle
        self.cfg = cfg
        c = ModelConfig(**cfg)
        self.ptr = oracle.lib.or_qmodel_synth(C.byref(c), seed, norm_jitter)
        if not self.ptr:
            raise ValueError("or_qmodel_synth: bits must be 4 or 8")

    def fill_kv(self, n, seed):
        self.o.lib.or_qmodel_fill_kv(self.ptr, n, seed)

    def set_len(self, n):
        """Rewind the cache to n positions (the next step writes position n)."""
        if self.o.lib.or_qmodel_set_len(self.ptr, int(n)) != n:
            raise ValueError("or_qmodel_set_len: n beyond the cache")

    def step(self, token):
        logits = np.empty(self.cfg["vocab"], np.float32)
        t = self.o.lib.or_qmodel_step(self.ptr, int(token), logits)
        if t < 0:
            raise RuntimeError("or_qmodel_step: cache full")
        return t, logits

    def close(self):
        if self.ptr:
            self.o.lib.or_qmodel_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.close()


def _dims(a):
    return np.ascontiguousarray(a.shape, np.uint64), a.ndim


class Reference:
    """The unmodified reference library (oracle/_ref/libti_ref.so) through ref_shim.cpp."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = self.lib = C.CDLL(path)
        L.ref_last_error.restype = C.c_char_p
        L.ref_matmul.argtypes = [_f32p, C.c_int, _u64p, _f32p, C.c_int, _u64p, _f32p]
        L.ref_rms_norm.argtypes = [_f32p, C.c_int, _u64p, _f32p, C.c_uint64, C.c_float, _f32p]
        L.ref_apply_rope.argtypes = [_f32p, C.c_int, _u64p, _f32p, C.c_int, _u64p, C.c_float, _f32p]
        for n in ("ref_silu", "ref_relu"):
            getattr(L, n).argtypes = [_f32p, C.c_uint64, _f32p]
        for n in ("ref_add", "ref_multiply"):
            getattr(L, n).argtypes = [_f32p, _f32p, C.c_uint64, _f32p]
        L.ref_softmax.argtypes = [_f32p, C.c_uint64, C.c_uint64, C.c_float, _f32p]
        L.ref_attention_fast_incremental.argtypes = [_f32p, _f32p, _f32p, C.c_uint64, C.c_uint64, C.c_uint64, _f32p]
        L.ref_multi_head_attention.argtypes = [_f32p, _f32p, _f32p] + [C.c_uint64] * 4 + [_f32p]
        L.ref_attention_general.argtypes = [_f32p, _f32p, _f32p, C.c_void_p] + [C.c_uint64] * 5 + [_f32p]
        L.ref_quantize.argtypes = [_f32p, C.c_uint64, C.c_int, C.c_int, _i32p, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.ref_dequantize.argtypes = [_i32p, C.c_uint64, C.c_int, C.c_float, C.c_float, _f32p]
        L.ref_plumbing_generate.argtypes = [C.c_uint64] * 3 + [_i32p, C.c_uint64, C.c_uint64, _i32p, C.POINTER(C.c_uint64)]
        L.ref_plumbing_generate_cfg.argtypes = [C.c_uint64] * 3 + [_i32p, C.c_uint64, C.c_uint64, C.c_int32, C.c_uint64,
                                                _i32p, C.POINTER(C.c_uint64), C.POINTER(C.c_int32),
                                                C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.ref_plumbing_generate_sampled.argtypes = [C.c_uint64] * 3 + [_i32p, C.c_uint64, C.c_uint64, C.c_float,
                                                    C.c_uint64, C.c_float, _i32p, _f32p, C.POINTER(C.c_uint64)]
        L.ref_plumbing_beam_search.argtypes = [C.c_uint64] * 3 + [_i32p] + [C.c_uint64] * 3 + [
            C.c_float, C.c_uint64, C.c_float, C.c_float, _i32p, _i32p, _i32p, _f32p, C.POINTER(C.c_uint64)]
        L.ref_time_decode.argtypes = [C.c_uint64] * 5 + [C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]

    def _chk(self, rc):
        if rc < 0:
            raise RuntimeError(self.lib.ref_last_error().decode())
        return rc

    def matmul(self, a, b):
        a, b = f32(a), f32(b)
        ad, an = _dims(a)
        bd, bn = _dims(b)
        shape = a.shape[:-1] + (b.shape[-1],)
        y = np.empty(int(np.prod(shape)), np.float32)
        self._chk(self.lib.ref_matmul(a.reshape(-1), an, ad, b.reshape(-1), bn, bd, y))
        return y.reshape(shape)

    def rms_norm(self, x, w, eps=1e-5):
        x, w = f32(x), f32(w)
        xd, xn = _dims(x)
        y = np.empty(x.size, np.float32)
        self._chk(self.lib.ref_rms_norm(x.reshape(-1), xn, xd, w, w.size, eps, y))
        return y.reshape(x.shape)

    def apply_rope(self, x, pos, theta=10000.0):
        x, pos = f32(x), f32(pos)
        xd, xn = _dims(x)
        pd, pn = _dims(pos)
        y = np.empty(x.size, np.float32)
        self._chk(self.lib.ref_apply_rope(x.reshape(-1), xn, xd, pos.reshape(-1), pn, pd, theta, y))
        return y.reshape(x.shape)

    def _unary(self, name, x):
        x = f32(x)
        y = np.empty(x.size, np.float32)
        self._chk(getattr(self.lib, name)(x.reshape(-1), x.size, y))
        return y.reshape(x.shape)

    def silu(self, x):
        return self._unary("ref_silu", x)

    def relu(self, x):
        return self._unary("ref_relu", x)

    def add(self, a, b):
        a, b = f32(a), f32(b)
        y = np.empty(a.size, np.float32)
        self._chk(self.lib.ref_add(a.reshape(-1), b.reshape(-1), a.size, y))
        return y.reshape(a.shape)

    def multiply(self, a, b):
        a, b = f32(a), f32(b)
        y = np.empty(a.size, np.float32)
        self._chk(self.lib.ref_multiply(a.reshape(-1), b.reshape(-1), a.size, y))
        return y.reshape(a.shape)

    def softmax(self, x, temperature=1.0):
        x = f32(x)
        n = x.shape[-1]
        y = np.empty(x.size, np.float32)
        self._chk(self.lib.ref_softmax(x.reshape(-1), x.size // n, n, temperature, y))
        return y.reshape(x.shape)

    def attention_incremental(self, q, k, v):
        q, k, v = f32(q), f32(k), f32(v)
        B, S, D = k.shape
        y = np.empty(B * D, np.float32)
        self._chk(self.lib.ref_attention_fast_incremental(q.reshape(-1), k.reshape(-1), v.reshape(-1), B, S, D, y))
        return y.reshape(B, 1, D)

    def attention_general(self, q, k, v, heads=0, mask=None):
        """TensorEngine::attention (heads 0) / multi_head_attention, any query length, optional mask."""
        q, k, v = f32(q), f32(k), f32(v)
        B, Sq, H = q.shape
        Sk = k.shape[1]
        m = None if mask is None else f32(mask).reshape(-1)
        y = np.empty(B * Sq * H, np.float32)
        self._chk(self.lib.ref_attention_general(q.reshape(-1), k.reshape(-1), v.reshape(-1),
                                                 None if m is None else m.ctypes.data, B, Sq, Sk, H, heads, y))
        return y.reshape(B, Sq, H)

    def multi_head_attention(self, q, k, v, heads):
        q, k, v = f32(q), f32(k), f32(v)
        B, S, H = k.shape
        y = np.empty(B * H, np.float32)
        self._chk(self.lib.ref_multi_head_attention(q.reshape(-1), k.reshape(-1), v.reshape(-1), B, S, H, heads, y))
        return y.reshape(B, 1, H)

    def quantize(self, x, bits, symmetric=True):
        x = f32(x).reshape(-1)
        q = np.empty(x.size, np.int32)
        s, z = C.c_float(), C.c_float()
        self._chk(self.lib.ref_quantize(x, x.size, bits, int(symmetric), q, C.byref(s), C.byref(z)))
        return q, s.value, z.value

    def dequantize(self, q, bits, scale, zp):
        q = np.ascontiguousarray(q, np.int32).reshape(-1)
        y = np.empty(q.size, np.float32)
        self._chk(self.lib.ref_dequantize(q, q.size, bits, scale, zp, y))
        return y

    def plumbing_generate(self, vocab, hidden, layers, prompt, max_new):
        p = np.ascontiguousarray(prompt, np.int32)
        out = np.zeros(len(prompt) + max_new + 1, np.int32)
        n = C.c_uint64()
        self._chk(self.lib.ref_plumbing_generate(vocab, hidden, layers, p, p.size, max_new, out, C.byref(n)))
        return out[: n.value].tolist()

    def plumbing_generate_cfg(self, vocab, hidden, layers, prompt, max_new, eos_token_id, max_len):
        """The reference's greedy generate() with config.eos_token_id / max_sequence_length set:
        (tokens, finished, stop code 0 eos_token / 1 max_length / 2 max_new_tokens, total_time_ms,
        tokens_per_second)."""
        p = np.ascontiguousarray(prompt, np.int32)
        out = np.zeros(len(prompt) + max_new + 1, np.int32)
        n, stop, ms, tps = C.c_uint64(), C.c_int32(), C.c_float(), C.c_float()
        fin = self._chk(self.lib.ref_plumbing_generate_cfg(vocab, hidden, layers, p, p.size, max_new, eos_token_id,
                                                           max_len, out, C.byref(n), C.byref(stop), C.byref(ms),
                                                           C.byref(tps)))
        return out[: n.value].tolist(), bool(fin), stop.value, ms.value, tps.value

    def plumbing_generate_sampled(self, vocab, hidden, layers, prompt, max_new, temperature, top_k, top_p):
        """The reference's generate(..., include_logprobs=true) with a sampling config: (all
        tokens, log-prob of each sampled token)."""
        p = np.ascontiguousarray(prompt, np.int32)
        out = np.zeros(len(prompt) + max_new + 1, np.int32)
        lp = np.zeros(max_new + 1, np.float32)
        n = C.c_uint64()
        k = self.lib.ref_plumbing_generate_sampled(vocab, hidden, layers, p, p.size, max_new, temperature, top_k,
                                                   top_p, out, lp, C.byref(n))
        self._chk(k)
        return out[: n.value].tolist(), lp[:k].copy()

    def plumbing_beam_search(self, vocab, hidden, layers, prompt, max_new, beam, temperature, top_k, top_p,
                             length_penalty):
        """The reference's generate_beam_search(include_logprobs=true): [(new tokens, finished,
        per-token log-prob)] in result order."""
        p = np.ascontiguousarray(prompt, np.int32)
        toks = np.zeros(beam * max_new, np.int32)
        nt, fin = np.zeros(beam, np.int32), np.zeros(beam, np.int32)
        lp = np.zeros(beam, np.float32)
        n = C.c_uint64()
        self._chk(self.lib.ref_plumbing_beam_search(vocab, hidden, layers, p, p.size, max_new, beam, temperature,
                                                    top_k, top_p, length_penalty, toks, nt, fin, lp, C.byref(n)))
        return [(toks[r * max_new: r * max_new + nt[r]].tolist(), bool(fin[r]), float(lp[r])) for r in range(n.value)]

    def time_decode(self, H, heads, inter, vocab, L, weight_kind=1, n_layers=1):
        ls, hs = C.c_double(), C.c_double()
        self._chk(self.lib.ref_time_decode(H, heads, inter, vocab, L, weight_kind, n_layers, C.byref(ls), C.byref(hs)))
        return ls.value, hs.value
