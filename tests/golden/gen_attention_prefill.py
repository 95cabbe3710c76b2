"""Golden vectors for TensorEngine::attention / multi_head_attention with query length > 1 and a
mask (tensor_engine.cpp:1045-1147, 1149-1252), from the COMPILED REFERENCE (oracle/_ref via
oracle/ref_shim.cpp ref_attention_general).  Build container only:

    make -C oracle ref && python tests/golden/gen_attention_prefill.py

Writes tests/golden/attention_prefill.npz (inputs + expected outputs) and its manifest entry.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "..", "oracle"))
from pyoracle import Reference  # noqa: E402

f32 = np.float32
ref = Reference()
# (B, Sq, Sk, H, heads (0 = TensorEngine::attention), mask kind)
CASES = [(1, 4, 16, 64, 0, "causal"), (2, 8, 24, 128, 4, "random"), (1, 16, 32, 256, 4, "none"),
         (1, 5, 13, 64, 2, "causal"), (3, 7, 40, 96, 3, "random"), (1, 1, 9, 64, 2, "random")]
cases = {}
for i, (B, Sq, Sk, H, heads, kind) in enumerate(CASES):
    rs = np.random.RandomState(1200 + i)
    q = rs.standard_normal((B, Sq, H)).astype(f32)
    k = rs.standard_normal((B, Sk, H)).astype(f32)
    v = rs.standard_normal((B, Sk, H)).astype(f32)
    if kind == "causal":   # query j sees keys [0, Sk - Sq + j]
        mask = np.tril(np.ones((Sq, Sk), f32), Sk - Sq)[None].repeat(B, 0)
    elif kind == "random":
        mask = (rs.uniform(size=(B, Sq, Sk)) < 0.7).astype(f32)
        mask[..., 0] = 1.0
    else:
        mask = None
    cases[f"shape{i}"] = np.array([B, Sq, Sk, H, heads])
    cases[f"q{i}"], cases[f"k{i}"], cases[f"v{i}"] = q, k, v
    if mask is not None:
        cases[f"mask{i}"] = mask
    cases[f"y{i}"] = ref.attention_general(q, k, v, heads, mask)
path = os.path.join(HERE, "attention_prefill.npz")
np.savez_compressed(path, **cases)
man = os.path.join(HERE, "manifest.json")
m = json.load(open(man))
m["files"]["attention_prefill.npz"] = ("TensorEngine::attention / multi_head_attention with query length > 1 and "
                                       "masks (tests/golden/gen_attention_prefill.py); q,k,v = RandomState(1200+i)")
json.dump(m, open(man, "w"), indent=1)
print(f"wrote attention_prefill.npz ({os.path.getsize(path) // 1024} KiB)")
