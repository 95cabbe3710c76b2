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
