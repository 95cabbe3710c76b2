"""Time ti_attn_prefill alone (HIP events, 50 launches): a 7B prompt chunk (32 heads, hd 128)
of M rows at positions 0..M-1, and the same chunk through ti_attn_decode (stride 0)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

T.init(0)
L = T.lib()
L.ti_event_elapsed_ms.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_float)]
a, b = C.c_void_p(), C.c_void_p()
T.check(L.ti_event_create(C.byref(a)))
T.check(L.ti_event_create(C.byref(b)))
heads, hd, max_seq = 32, 128, 2048
rng = np.random.RandomState(0)
for kvh, M in [(32, 128), (32, 256), (32, 512), (32, 1024), (8, 512)]:   # 7B MHA; Llama-3-8B GQA 4
    kc = T.DeviceBuffer.from_array(rng.standard_normal((kvh, max_seq, hd)).astype(np.float16))
    vc = T.DeviceBuffer.from_array(rng.standard_normal((kvh, max_seq, hd)).astype(np.float16))
    q = T.DeviceBuffer.from_array(rng.standard_normal((M, heads * hd)).astype(np.float32))
    pos = T.DeviceBuffer.from_array(np.arange(M, dtype=np.int32))
    out = T.DeviceBuffer(M * heads * hd * 2)
    ws = T.DeviceBuffer(L.ti_attn_workspace_bytes(M, heads, hd, 4))
    ws.zero()
    runs = {"prefill": lambda: L.ti_attn_prefill(q.ptr, kc.ptr, vc.ptr, max_seq, pos.ptr, M, heads, kvh, hd, out.ptr, None),
            "decode": lambda: L.ti_attn_decode(q.ptr, kc.ptr, vc.ptr, 0, max_seq, pos.ptr, M, heads, kvh, hd, 4, ws.ptr,
                                               out.ptr, None)}
    for name, f in runs.items():
        T.check(f())
        T.check(L.ti_event_record(a, None))
        for _ in range(50):
            f()
        T.check(L.ti_event_record(b, None))
        ms = C.c_float()
        T.check(L.ti_event_elapsed_ms(a, b, C.byref(ms)))
        print(f"M {M:5d} kv_heads {kvh:2d} {name:8s}: {ms.value * 1e3 / 50:8.1f} us per launch", flush=True)
