"""the device sampler's large-k path (top_k > TI_SAMPLE_MAX_K: keys and sort in an HBM
workspace) against the host path the C++ API would otherwise take for one request (logits to the
host + ti_sample_token, the reference's std::sort over all V).  Device: HIP events over 50
launches of ti_sample_device_ws; host: wall time of the D2H copy + ti_sample_token."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

T.init(0)
L = T.lib()
L.ti_event_elapsed_ms.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_float)]
for V, k, p in [(128256, 4096, 0.9), (128256, 8192, 0.9), (128256, 65536, 0.9), (128256, 128256, 1.0),
                (128256, 128256, 0.9), (32000, 32000, 0.9)]:
    host_lg = (np.random.RandomState(0).standard_normal(V) * 3).astype(np.float32)
    lg = T.DeviceBuffer.from_array(host_lg)
    dr = T.DeviceBuffer.from_array(np.array([0.3], np.float32))
    tok = T.DeviceBuffer(4)
    wsb = L.ti_sample_workspace_bytes(V, k)
    ws = T.DeviceBuffer(max(wsb, 16))
    a, b = C.c_void_p(), C.c_void_p()
    T.check(L.ti_event_create(C.byref(a)))
    T.check(L.ti_event_create(C.byref(b)))
    T.check(L.ti_sample_device_ws(lg.ptr, V, 1, V, 0.8, k, p, dr.ptr, tok.ptr, None, None, ws.ptr))
    T.check(L.ti_event_record(a, None))
    for _ in range(50):
        L.ti_sample_device_ws(lg.ptr, V, 1, V, 0.8, k, p, dr.ptr, tok.ptr, None, None, ws.ptr)
    T.check(L.ti_event_record(b, None))
    ms = C.c_float()
    T.check(L.ti_event_elapsed_ms(a, b, C.byref(ms)))
    dev_us = ms.value * 1e3 / 50
    T.sync()
    t0 = time.perf_counter()
    for _ in range(5):
        h = lg.download(np.float32, (V,))
        T.sample_token(h, 0.8, k, p, 0.3)
    host_us = (time.perf_counter() - t0) / 5 * 1e6
    print(f"V {V:6d} top_k {k:6d} top_p {p}: device {dev_us:8.1f} us, host (D2H + ti_sample_token) {host_us:9.1f} us",
          flush=True)
