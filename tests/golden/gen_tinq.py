"""TINQ fixtures from the COMPILED REFERENCE (build container only: oracle/_ref/libti_ref.so).

The reference's Quantizer::quantize_model + save_quantized_model
(src/optimize/quantization.cpp:79-211) on a small llama-named ModelData of seeded fp32
tensors; the fp32 inputs are stored next to the files (tinq_inputs.npz), so the C++ API's
own save can be compared byte for byte and its load checked field by field.

    python tests/golden/gen_tinq.py
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libti_ref.so")

# name order = insertion order (the reference's unordered_map then fixes the file order)
TENSORS = [("token_embeddings.weight", (64, 32)), ("layers.0.attention_norm.weight", (32,)),
           ("layers.0.attention.wq.weight", (32, 32)), ("layers.0.feed_forward.w1.weight", (32, 48)),
           ("norm.weight", (32,)), ("output.weight", (32, 64))]
META = dict(name="tinq_fixture", arch="llama", version="1.0", sizes=[64, 32, 1, 4, 48], rope_theta=10000.0)
CASES = {"tinq_int8_sym": (0, 1), "tinq_int4_sym": (1, 1), "tinq_int8_asym": (0, 0)}


def inputs():
    rng = np.random.RandomState(0x71E0)
    return {n: (rng.standard_normal(s) * 0.05).astype(np.float32) for n, s in TENSORS}


def main():
    L = C.CDLL(REF_SO)
    L.ref_last_error.restype = C.c_char_p
    x = inputs()
    np.savez_compressed(os.path.join(HERE, "tinq_inputs.npz"), **{n.replace(".", "__"): a for n, a in x.items()})
    n = len(TENSORS)
    names = (C.c_char_p * n)(*[t[0].encode() for t in TENSORS])
    arrs = [np.ascontiguousarray(x[t[0]]) for t in TENSORS]
    data = (C.c_void_p * n)(*[a.ctypes.data for a in arrs])
    ndims = (C.c_int * n)(*[a.ndim for a in arrs])
    dims = np.array([d for a in arrs for d in a.shape], np.uint64)
    sizes = np.array(META["sizes"], np.uint64)
    for case, (qtype, sym) in CASES.items():
        path = os.path.join(HERE, case + ".tinq")
        rc = L.ref_tinq_save(path.encode(), qtype, sym, n, names, data, ndims, dims.ctypes.data_as(C.c_void_p),
                             META["name"].encode(), META["arch"].encode(), META["version"].encode(),
                             sizes.ctypes.data_as(C.c_void_p), C.c_float(META["rope_theta"]))
        assert rc == 0, L.ref_last_error()
        print(case, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
