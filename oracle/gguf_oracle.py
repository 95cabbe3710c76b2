"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the GGUF v3 container and ggml's Q4_0 /
Q4_1 / Q8_0 block formats, the oracle for ModelLoader::load_gguf
(turboinfer_amd/csrc/api/gguf.cpp; reference src/model/model_loader.cpp:710-873).

* gguf_write: a GGUF v3 file (header, key/values, tensor infos, data at general.alignment).
  Quantizing writers follow ggml's reference quantizers (ggml-quants.c quantize_row_q4_0_ref,
  quantize_row_q4_1_ref, quantize_row_q8_0_ref: 32 weights per block, fp16 scale d, Q4_0
  d = signed max / -8 and q = min(15, trunc(x/d + 8.5)), Q4_1 d = (max - min) / 15, m = min and
  q = min(15, trunc((x - min)/d + 0.5)), Q8_0 d = amax / 127 and q = round(x/d)).
* gguf_read: the same file back, as the reference's ModelLoader maps it (metadata fields from
  the llama./gpt2. keys, every value as its std::to_string text, "[array]" for arrays, dims
  reversed to row-major), with the published layout where the reference mis-reads it
  (arrays walked, tensor i at data_start + offset_i, quantized blocks dequantized:
  y = (q - 8) d, q d + m, q d in fp32).

The reference itself pins the container walk on a file it reads correctly (scalar
key/values, one fp32 tensor): tests/test_cpp_api.py runs oracle/_ref's ModelLoader on
tests/golden/gguf_ref_pin.gguf.  The block formats are ggml's published ones (the
reference declares them fp32 and reads the packed bytes as floats, model_loader.cpp:165-182):
parity unpinned against the reference there, by construction.
"""
from __future__ import annotations

import struct

import numpy as np

MAGIC, VERSION = 0x46554747, 3
U8, I8, U16, I16, U32, I32, F32, BOOL, STR, ARR, U64, I64, F64 = range(13)
T_F32, T_F16, T_Q4_0, T_Q4_1, T_Q8_0, T_BF16 = 0, 1, 2, 3, 8, 30
_SCALAR = {U8: "<B", I8: "<b", U16: "<H", I16: "<h", U32: "<I", I32: "<i", F32: "<f", BOOL: "<B", U64: "<Q",
           I64: "<q", F64: "<d"}
_BLOCK = {T_Q4_0: 18, T_Q4_1: 20, T_Q8_0: 34}


# ------------------------------------------------------------------ quantizers (ggml reference)
def _blocks(x):
    x = np.asarray(x, np.float32).reshape(-1)
    assert x.size % 32 == 0
    return x.reshape(-1, 32)


def _trunc_i8(v):
    return np.trunc(v).astype(np.int32)


def quant_q8_0(x) -> bytes:
    out = bytearray()
    for b in _blocks(x):
        amax = np.float32(np.max(np.abs(b)))
        d = np.float32(amax / np.float32(127))
        idv = np.float32(1) / d if d != 0 else np.float32(0)
        v = (b * idv).astype(np.float32)
        q = (np.sign(v) * np.floor(np.abs(v) + np.float32(0.5))).astype(np.int8)   # roundf
        out += np.float16(d).tobytes() + q.tobytes()
    return bytes(out)


def quant_q4_0(x) -> bytes:
    out = bytearray()
    for b in _blocks(x):
        j = int(np.argmax(np.abs(b)))   # first index of the largest magnitude (strict < update)
        mx = b[j]
        d = np.float32(mx / np.float32(-8))
        idv = np.float32(1) / d if d != 0 else np.float32(0)
        x0 = (b[:16] * idv).astype(np.float32)
        x1 = (b[16:] * idv).astype(np.float32)
        q0 = np.minimum(15, _trunc_i8((x0 + np.float32(8.5)).astype(np.float32)))
        q1 = np.minimum(15, _trunc_i8((x1 + np.float32(8.5)).astype(np.float32)))
        out += np.float16(d).tobytes() + (q0 | (q1 << 4)).astype(np.uint8).tobytes()
    return bytes(out)


def quant_q4_1(x) -> bytes:
    out = bytearray()
    for b in _blocks(x):
        mn, mx = np.float32(np.min(b)), np.float32(np.max(b))
        d = np.float32((mx - mn) / np.float32(15))
        idv = np.float32(1) / d if d != 0 else np.float32(0)
        x0 = ((b[:16] - mn).astype(np.float32) * idv).astype(np.float32)
        x1 = ((b[16:] - mn).astype(np.float32) * idv).astype(np.float32)
        q0 = np.minimum(15, _trunc_i8((x0 + np.float32(0.5)).astype(np.float32)))
        q1 = np.minimum(15, _trunc_i8((x1 + np.float32(0.5)).astype(np.float32)))
        out += np.float16(d).tobytes() + np.float16(mn).tobytes() + (q0 | (q1 << 4)).astype(np.uint8).tobytes()
    return bytes(out)


def dequant(raw: bytes, ttype: int, n: int) -> np.ndarray:
    if ttype == T_F32:
        return np.frombuffer(raw, np.float32, n).copy()
    if ttype == T_F16:
        return np.frombuffer(raw, np.float16, n).copy()
    if ttype == T_BF16:
        return (np.frombuffer(raw, np.uint16, n).astype(np.uint32) << 16).view(np.float32)
    bs = _BLOCK[ttype]
    blk = np.frombuffer(raw, np.uint8).reshape(-1, bs)
    d = blk[:, 0:2].copy().view(np.float16).astype(np.float32)             # [nb, 1]
    if ttype == T_Q8_0:
        q = blk[:, 2:].view(np.int8).astype(np.float32)
        return (q * d).astype(np.float32).reshape(-1)
    qs = blk[:, (4 if ttype == T_Q4_1 else 2):]
    q = np.concatenate([qs & 0x0F, qs >> 4], axis=1).astype(np.int32)     # elements j, j + 16
    if ttype == T_Q4_0:
        return ((q - 8).astype(np.float32) * d).astype(np.float32).reshape(-1)
    m = blk[:, 2:4].copy().view(np.float16).astype(np.float32)
    return ((q.astype(np.float32) * d).astype(np.float32) + m).astype(np.float32).reshape(-1)


# ------------------------------------------------------------------------------- writer
def _str(s: str) -> bytes:
    b = s.encode()
    return struct.pack("<Q", len(b)) + b


def _value(vtype: int, v) -> bytes:
    if vtype == STR:
        return _str(v)
    if vtype == ARR:
        etype, items = v
        out = struct.pack("<IQ", etype, len(items))
        for it in items:
            out += _value(etype, it)
        return out
    return struct.pack(_SCALAR[vtype], v)


def gguf_write(path, kvs, tensors, alignment: int = 32) -> None:
    """kvs: [(key, vtype, value)] (ARR value = (elem_type, items)); tensors: [(name, array, ggml type)]."""
    head = struct.pack("<IIQQ", MAGIC, VERSION, len(tensors), len(kvs))
    for k, t, v in kvs:
        head += _str(k) + struct.pack("<I", t) + _value(t, v)
    blobs, off = [], 0
    for name, a, tt in tensors:
        a = np.asarray(a)
        raw = {T_F32: lambda x: np.asarray(x, np.float32).tobytes(), T_F16: lambda x: np.asarray(x, np.float16).tobytes(),
               T_BF16: lambda x: (np.asarray(x, np.float32).view(np.uint32) >> 16).astype(np.uint16).tobytes(),
               T_Q4_0: quant_q4_0, T_Q4_1: quant_q4_1, T_Q8_0: quant_q8_0}[tt](a)
        dims = list(reversed(a.shape))
        head += _str(name) + struct.pack("<I", len(dims)) + b"".join(struct.pack("<Q", d) for d in dims)
        head += struct.pack("<IQ", tt, off)
        blobs.append(raw)
        off += len(raw)
        off = (off + alignment - 1) // alignment * alignment
    pad = (-len(head)) % alignment
    data = bytearray()
    for raw in blobs:
        data += raw
        data += b"\0" * ((-len(data)) % alignment)
    with open(path, "wb") as f:
        f.write(head + b"\0" * pad + bytes(data))


# ------------------------------------------------------------------------------- reader
def _fmt_value(vtype: int, v) -> str:   # std::to_string / read_gguf_value (model_loader.cpp:60-153)
    if vtype in (F32, F64):
        return "%f" % v
    if vtype == BOOL:
        return "true" if v else "false"
    return str(v)


class _R:
    def __init__(self, b: bytes):
        self.b, self.p = b, 0

    def get(self, fmt):
        v = struct.unpack_from(fmt, self.b, self.p)[0]
        self.p += struct.calcsize(fmt)
        return v

    def str(self):
        n = self.get("<Q")
        s = self.b[self.p:self.p + n].decode()
        self.p += n
        return s

    def value(self, t):
        if t == STR:
            return self.str()
        if t == ARR:
            et, n = self.get("<I"), self.get("<Q")
            return [self.value(et) for _ in range(n)]
        return self.get(_SCALAR[t])


def gguf_read(path):
    """-> (meta [name, arch, version, vocab, hidden, layers, heads, inter, rope], extras {k: text},
    {name: (dtype code 0 f32 / 3 f16, shape, array)}) as ModelLoader::load maps the file."""
    b = open(path, "rb").read()
    r = _R(b)
    magic, version, nt, nkv = r.get("<I"), r.get("<I"), r.get("<Q"), r.get("<Q")
    assert magic == MAGIC and version == VERSION
    import os
    meta = [os.path.splitext(os.path.basename(path))[0], "unknown", "gguf_v%d" % version, 0, 0, 0, 0, 0,
            np.float32(10000.0)]
    extras, alignment = {}, 32
    fields = {"general.architecture": 1, "general.name": 0, "llama.vocab_size": 3, "gpt2.vocab_size": 3,
              "llama.embedding_length": 4, "gpt2.embedding_length": 4, "llama.block_count": 5, "gpt2.block_count": 5,
              "llama.attention.head_count": 6, "gpt2.attention.head_count": 6, "llama.feed_forward_length": 7,
              "gpt2.feed_forward_length": 7, "llama.rope.theta": 8}
    for _ in range(nkv):
        k, t = r.str(), r.get("<I")
        v = r.value(t)
        text = "[array]" if t == ARR else _fmt_value(t, v)
        if k == "general.alignment" and t == U32:
            alignment = v
        if k in fields:
            i = fields[k]
            meta[i] = text if i < 3 else (np.float32(float(text)) if i == 8 else int(text))
        else:
            extras[k] = text
    infos = []
    for _ in range(nt):
        name = r.str()
        nd = r.get("<I")
        dims = [r.get("<Q") for _ in range(nd)]
        tt, off = r.get("<I"), r.get("<Q")
        infos.append((name, tuple(reversed(dims)), tt, off))
    start = (r.p + alignment - 1) // alignment * alignment
    tensors = {}
    for name, shape, tt, off in infos:
        n = int(np.prod(shape))
        nbytes = {T_F32: 4 * n, T_F16: 2 * n, T_BF16: 2 * n}.get(tt) or n // 32 * _BLOCK[tt]
        arr = dequant(b[start + off:start + off + nbytes], tt, n).reshape(shape)
        tensors[name] = (3 if tt == T_F16 else 0, shape, arr)
    return meta, extras, tensors
