"""Microbenchmark of ti_gemm_wq_a16 on the Llama-2-7B decode shapes (GPU box).

    python tools/gemv_sweep.py [reps]

Times back-to-back launches between HIP events for each (shape, x_kind) and prints GB/s of
algorithmic bytes (packed weights + scales + activations).  Run under different
TI_GEMV_WG_PER_CU values to compare grid sizes."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
T.init(0)
L = T.lib()
shapes = [("qkv", 4096, 12288), ("o", 4096, 4096), ("gate_up", 4096, 22016), ("down", 11008, 4096),
          ("lm_head", 4096, 32000)]
ev0, ev1 = C.c_void_p(), C.c_void_p()
T.check(L.ti_event_create(C.byref(ev0)))
T.check(L.ti_event_create(C.byref(ev1)))
for M in (1,):
    for name, K, N in shapes:
        tb, sb = L.ti_wpack_tile_bytes(4, K, N), L.ti_wpack_scale_bytes(4, K, N)
        tiles, scales = T.DeviceBuffer(tb), T.DeviceBuffer(sb)
        T.check(L.ti_wsynth_device(1, 7, K, N, N, 4, 0, 0, tiles.ptr, scales.ptr, None))
        x32 = T.DeviceBuffer.from_array(np.random.RandomState(0).standard_normal((M, K)).astype(np.float32))
        x16 = T.DeviceBuffer.from_array(np.random.RandomState(0).standard_normal((M, K)).astype(np.float16))
        nw = T.DeviceBuffer.from_array(np.ones(K, np.float32))
        y = T.DeviceBuffer(M * N * 4)
        ep = T.Epilogue()
        ep.kind, ep.ldo, ep.out = T.EPI_STORE_F32, N, y.ptr
        for xk, xd in ((T.X_F16, x16), (T.X_F32_RMSNORM, x32)):
            def run():
                T.check(L.ti_gemm_wq_a16(tiles.ptr, scales.ptr, 4, xd.ptr, xk, K, nw.ptr, 1e-5, M, N, K,
                                         C.byref(ep), None))
            run()
            T.sync()
            T.check(L.ti_event_record(ev0, None))
            for _ in range(reps):
                run()
            T.check(L.ti_event_record(ev1, None))
            ms = C.c_float()
            T.check(L.ti_event_elapsed_ms(ev0, ev1, C.byref(ms)))
            us = ms.value * 1e3 / reps
            by = tb + sb + M * K * (2 if xk == T.X_F16 else 4)
            print(f"M={M} {name:8s} K={K:6d} N={N:6d} x={'f16 ' if xk == T.X_F16 else 'norm'} "
                  f"{us:8.2f} us  {by / us / 1e3:8.1f} GB/s", flush=True)
