"""The CPU oracle (oracle/ti_oracle.c) against golden vectors produced by the compiled
reference (tests/golden/gen_golden.py).  Bit-exact: the oracle restates the reference build's
rounding sequence, so every float must match to the last bit."""
from __future__ import annotations

import hashlib
import json

import numpy as np
import pytest

from conftest import inp


def same_bits(y, d, key):
    y = np.ascontiguousarray(y, np.float32)
    if key in d:
        exp = d[key]
        assert y.shape == exp.shape or y.size == exp.size
        np.testing.assert_array_equal(y.reshape(-1).view(np.uint32), exp.reshape(-1).view(np.uint32))
    else:
        head = d[key + "_head"]
        np.testing.assert_array_equal(y.reshape(-1)[: head.size].view(np.uint32), head.view(np.uint32))
        assert hashlib.sha256(y.tobytes()).digest() == d[key + "_sha"].tobytes()


def ncases(d, prefix="shape"):
    return len([k for k in d.files if k.startswith(prefix)])


def test_matmul(oracle, golden):
    d = golden("matmul")
    for i in range(ncases(d)):
        B, M, K, N = d[f"shape{i}"]
        sa, sb = d[f"seeds{i}"]
        a, b = inp(int(sa), (B, M, K)), inp(int(sb), (K, N), 0.05)
        same_bits(oracle.matmul(a, b), d, f"y{i}")


def test_rms_norm(oracle, golden):
    d = golden("rms_norm")
    for i in range(ncases(d)):
        rows, n = d[f"shape{i}"]
        x = inp(200 + i, (rows, n))
        w = (np.float32(1.0) + inp(300 + i, (n,), 0.1)).astype(np.float32)
        same_bits(oracle.rms_norm(x, w), d, f"y{i}")


def test_rope(oracle, golden):
    d = golden("rope")
    for i in range(ncases(d)):
        shape = tuple(int(s) for s in d[f"shape{i}"])
        x = inp(400 + i, shape)
        same_bits(oracle.apply_rope(x, d[f"pos{i}"], float(d[f"theta{i}"][0])), d, f"y{i}")


def test_eltwise(oracle, golden):
    d = golden("eltwise")
    x, x2 = inp(500, (1001,), 4.0), inp(501, (1001,))
    same_bits(oracle.silu(x), d, "silu")
    same_bits(oracle.relu(x), d, "relu")
    same_bits(oracle.add(x, x2), d, "add")
    same_bits(oracle.multiply(x, x2), d, "mul")


def test_softmax(oracle, golden):
    d = golden("softmax")
    for i in range(ncases(d)):
        rows, n = d[f"shape{i}"]
        x = inp(600 + i, (rows, n), 5.0)
        same_bits(oracle.softmax(x, float(d[f"T{i}"][0])), d, f"y{i}")


def test_attention_incremental(oracle, golden):
    d = golden("attention")
    for i in range(ncases(d)):
        B, S, D = (int(v) for v in d[f"shape{i}"])
        q, k, v = inp(700 + 3 * i, (B, 1, D)), inp(701 + 3 * i, (B, S, D)), inp(702 + 3 * i, (B, S, D))
        same_bits(oracle.attention_incremental(q, k, v), d, f"y{i}")


def test_multi_head_attention(oracle, golden):
    d = golden("mha")
    for i in range(ncases(d)):
        S, H, heads = (int(v) for v in d[f"shape{i}"])
        q, k, v = inp(800 + 3 * i, (1, 1, H)), inp(801 + 3 * i, (1, S, H)), inp(802 + 3 * i, (1, S, H))
        same_bits(oracle.multi_head_attention(q, k, v, heads), d, f"y{i}")


def test_quantization(oracle, golden):
    d = golden("quant")
    for k in range(int(d["n"][0])):
        x, bits, sym = d[f"x{k}"], int(d[f"bits{k}"][0]), bool(d[f"sym{k}"][0])
        s, z = oracle.quant_info(x, bits, sym)
        assert np.float32(s).view(np.uint32) == d[f"scale{k}"].view(np.uint32)[0]
        assert np.float32(z).view(np.uint32) == d[f"zp{k}"].view(np.uint32)[0]
        q = oracle.quantize(x, bits, s, z)
        np.testing.assert_array_equal(q, d[f"q{k}"])
        same_bits(oracle.dequantize(q, bits, s, z), d, f"deq{k}")


def test_quantization_roundtrip_bounds(oracle):
    """The reference's own acceptance bound (tests/test_quantization_complete.cpp:20-131):
    symmetric round-trip error < 1.0 on its grids."""
    for bits, x in ((8, np.linspace(-10, 10, 16)), (4, np.linspace(-2, 2, 9))):
        x = x.astype(np.float32)
        s, z = oracle.quant_info(x, bits, True)
        y = oracle.dequantize(oracle.quantize(x, bits, s, z), bits, s, z)
        assert np.max(np.abs(y - x)) < 1.0


def test_plumbing_generate(oracle, golden):
    d = golden("plumbing_generate")
    for i in range(3):
        toks, _ = oracle.plumbing_generate(1000, 256, 4, d[f"prompt{i}"].tolist(), 20)
        assert toks == d[f"tokens{i}"].tolist()


def test_generate_contract_oracle(oracle, golden):
    """The oracle's generate loop stops as the compiled reference does (gen_generate_contract.py):
    on token id 2 (the config's eos_token_id is not consulted, inference_engine.cpp:759-760) or at
    max_sequence_length (:767)."""
    d = golden("generate_contract")
    for i in range(int(d["n"][0])):
        V, H, layers, max_new, _eos, max_len = (int(v) for v in d[f"cfg{i}"])
        toks, _ = oracle.plumbing_generate(V, H, layers, d[f"prompt{i}"].tolist(), max_new, max_seq=max_len)
        assert toks == d[f"tokens{i}"].tolist(), i


@pytest.mark.parametrize("name", ["mini_gqa_w4", "mini_hd128_w8"])
def test_decode_step_reference_composed(oracle, golden, name):
    """or_decode_step (fp32 cache) == the decode step composed from reference ops."""
    from pyoracle import OracleModel
    d = golden(f"decode_{name}")
    cfg = json.loads(str(d["cfg"]))
    m = OracleModel(oracle, cfg, int(d["seed"][0]), float(d["jitter"][0]))
    toks = d["tokens"].tolist()
    n_prompt = d["prompt"].size
    logits_all = []
    produced = []
    for pos in range(len(toks) - 1):
        t, lg = m.step(toks[pos], kv_round_f16=False)
        logits_all.append(lg)
        if pos >= n_prompt - 1:
            produced.append(t)
    np.testing.assert_array_equal(np.stack(logits_all).view(np.uint32), d["logits"].view(np.uint32))
    assert produced == toks[n_prompt:]
    m.close()


def test_sampler_greedy_matches_argmax(oracle):
    rng = np.random.RandomState(3)
    for _ in range(20):
        lg = rng.standard_normal(1000).astype(np.float32)
        t, _ = oracle.sample_token(lg, 1.0, 1, 0.9, 0.5)
        assert t == int(np.argmax(lg))
