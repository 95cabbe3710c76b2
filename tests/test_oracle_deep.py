"""The full-depth oracle (oracle/ti_oracle_deep.c) is the pinned oracle's decode step:
bit-identical logits and tokens to OracleModel.step (or_decode_step, itself pinned to the
compiled reference's composed decode by test_oracle_golden.py) on the same synthetic model, KV
fill and tokens.  The full-depth fixtures (tests/golden/gen_deep.py) are made with it."""
from __future__ import annotations

import numpy as np
import pytest

from pyoracle import OracleDeepModel, OracleModel

CASES = {
    "gqa_w4": dict(vocab=700, hidden=256, layers=3, heads=8, kv_heads=2, head_dim=32, inter=384,
                   rope_theta=10000.0, eps=1e-5, bits=4, group=128, max_seq=96),
    "hd128_w8": dict(vocab=300, hidden=384, layers=2, heads=3, kv_heads=3, head_dim=128, inter=640,
                     rope_theta=500000.0, eps=1e-5, bits=8, group=128, max_seq=64),
    "hd64_w8_gqa4": dict(vocab=512, hidden=512, layers=2, heads=8, kv_heads=2, head_dim=64, inter=768,
                         rope_theta=10000.0, eps=1e-5, bits=8, group=128, max_seq=80),
}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("jitter", [0.0, 0.1])
def test_deep_oracle_bit_identical_to_decode_step(oracle, name, jitter):
    cfg = CASES[name]
    seed, fill, kv_seed = 41, cfg["max_seq"] - 5, 9
    a = OracleModel(oracle, cfg, seed, jitter)
    b = OracleDeepModel(oracle, cfg, seed, jitter)
    a.fill_kv(fill, kv_seed)
    b.fill_kv(fill, kv_seed)
    tok = 7
    for _ in range(5):
        ta, la = a.step(tok)
        tb, lb = b.step(tok)
        np.testing.assert_array_equal(la.view(np.uint32), lb.view(np.uint32))
        assert ta == tb
        tok = ta
    with pytest.raises(RuntimeError):
        b.step(tok)
    a.close()
    b.close()


def test_long_fixture_consistent_and_reproduced(oracle, golden):
    """tests/golden/deep_long_tinyllama_1b.npz (gen_deep_long.py): the stored top-k, margins and
    full logits agree with each other, and the oracle reproduces its first steps bit for bit."""
    import json
    d = golden("deep_long_tinyllama_1b")
    cfg = json.loads(str(d["cfg"]))
    top_i, top_v, toks = d["top_idx"], d["top_val"], d["tokens"]
    np.testing.assert_array_equal(top_i[:, 0], toks)
    np.testing.assert_array_equal(d["margin"], top_v[:, 0] - top_v[:, 1])
    for i, s in enumerate(d["full_at"]):
        np.testing.assert_array_equal(d["full_logits"][i][top_i[s]], top_v[s])
        assert float(np.abs(d["full_logits"][i]).max()) == float(d["maxabs"][s])
    m = OracleDeepModel(oracle, cfg, int(d["seed"][0]), 0.0)
    m.fill_kv(int(d["fill"][0]), int(d["stream"][1]))
    t = int(d["stream"][0])
    for step in range(2):
        t, lg = m.step(t)
        assert t == toks[step]
        np.testing.assert_array_equal(lg.view(np.uint32), d["full_logits"][step].view(np.uint32))
    m.close()
