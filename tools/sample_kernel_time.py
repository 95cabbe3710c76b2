"""Time ti_sample_device alone (HIP events, 200 launches) for a few vocab sizes / top-k."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

T.init(0)
L = T.lib()
for V, k, p in [(32000, 40, 0.9), (32000, 40, 1.0), (32000, 1024, 0.9), (128256, 40, 0.9), (32000, 2048, 1.0),
                (32000, 4096, 0.9), (128256, 4096, 0.9)]:
    lg = T.DeviceBuffer.from_array((np.random.RandomState(0).standard_normal(V) * 3).astype(np.float32))
    dr = T.DeviceBuffer.from_array(np.array([0.3], np.float32))
    tok = T.DeviceBuffer(4)
    a, b = C.c_void_p(), C.c_void_p()
    T.check(L.ti_event_create(C.byref(a)))
    T.check(L.ti_event_create(C.byref(b)))
    T.check(L.ti_sample_device(lg.ptr, V, 1, V, 0.8, k, p, dr.ptr, tok.ptr, None, None))
    T.check(L.ti_event_record(a, None))
    for _ in range(200):
        L.ti_sample_device(lg.ptr, V, 1, V, 0.8, k, p, dr.ptr, tok.ptr, None, None)
    T.check(L.ti_event_record(b, None))
    ms = C.c_float()
    L.ti_event_elapsed_ms.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_float)]
    T.check(L.ti_event_elapsed_ms(a, b, C.byref(ms)))
    print(f"V {V:6d} top_k {k:4d} top_p {p}: {ms.value * 1e3 / 200:7.1f} us per sample", flush=True)
