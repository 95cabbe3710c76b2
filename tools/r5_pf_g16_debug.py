"""Debug: which outputs of ti_attn_prefill are non-finite at heads / kv_heads = 16 (each kernel forced)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

T.init(0)
L = T.lib()
for (M, nh, nkv, start, max_seq) in [(77, 32, 2, 3, 96), (77, 32, 4, 3, 96), (64, 16, 1, 0, 64)]:
    rng = np.random.RandomState(1)
    hd = 128
    kc = rng.standard_normal((nkv, max_seq, hd)).astype(np.float16)
    vc = rng.standard_normal((nkv, max_seq, hd)).astype(np.float16)
    pos = (start + np.arange(M)).astype(np.int32)
    kc[:, pos.max() + 1:] = np.nan
    vc[:, pos.max() + 1:] = np.nan
    q = rng.standard_normal((M, nh * hd)).astype(np.float32)
    kd, vd, qd, pd = (T.DeviceBuffer.from_array(a) for a in (kc, vc, q, pos))
    for mode in (1, 2, 3):
        L.ti_attn_prefill_set_kernel(mode)
        out = T.DeviceBuffer(M * nh * hd * 2)
        T.check(L.ti_attn_prefill(qd.ptr, kd.ptr, vd.ptr, max_seq, pd.ptr, M, nh, nkv, hd, out.ptr, None))
        T.sync()
        o = out.download(np.float16, (M, nh, hd)).astype(np.float32)
        bad = ~np.isfinite(o)
        rows = np.unique(np.nonzero(bad)[0])
        heads = np.unique(np.nonzero(bad)[1])
        print(f"M {M} nh {nh} nkv {nkv} mode {mode}: non-finite {bad.sum()} rows {rows[:10]} heads {heads[:10]}", flush=True)
    L.ti_attn_prefill_set_kernel(0)
