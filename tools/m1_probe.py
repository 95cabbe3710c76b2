"""One-row (decode) fused-GEMV launch time against shape: how much of a launch is fixed cost and
how much follows the bytes a workgroup streams (GPU box, diagnostic only).

    python tools/m1_probe.py

Cold weights (launches cycle through enough copies to exceed the 256 MiB Infinity Cache), fp16 x,
plain fp32 store epilogue, back-to-back launches on one stream between HIP events.  Prints us per
launch, the workgroup count and KiB streamed per workgroup, for the TinyLlama INT8 and Llama-2-7B
INT4 projections and for variants with K halved (same grid, half the bytes per workgroup) or N
doubled (twice the grid)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

T.init(0)
L = T.lib()
shapes = [
    (8, "tl qkv", 2048, 2560), (8, "tl o", 2048, 2048), (8, "tl o k/2", 1024, 2048), (8, "tl o 2n", 2048, 4096),
    (8, "tl gate_up", 2048, 11264), (8, "tl down", 5632, 2048), (8, "tl down k/2", 2816, 2048),
    (8, "tl down 2n", 5632, 4096),
    (4, "7b qkv", 4096, 12288), (4, "7b o", 4096, 4096), (4, "7b o k/2", 2048, 4096), (4, "7b gate_up", 4096, 22016),
    (4, "7b down", 11008, 4096), (4, "7b down k/2", 5504, 4096), (4, "7b down 2n", 11008, 8192),
]
ev0, ev1 = C.c_void_p(), C.c_void_p()
T.check(L.ti_event_create(C.byref(ev0)))
T.check(L.ti_event_create(C.byref(ev1)))
for bits, name, K, N in shapes:
    tb, sb = L.ti_wpack_tile_bytes(bits, K, N), L.ti_wpack_scale_bytes(bits, K, N)
    copies = max(2, int(320e6 // (tb + sb)) + 1)
    W = []
    for c in range(copies):
        tiles, scales = T.DeviceBuffer(tb), T.DeviceBuffer(sb)
        T.check(L.ti_wsynth_device(1, 7 + c, K, N, N, bits, 0, 0, tiles.ptr, scales.ptr, None))
        W.append((tiles, scales))
    x16 = T.DeviceBuffer.from_array(np.random.RandomState(0).standard_normal((1, K)).astype(np.float16))
    y = T.DeviceBuffer(N * 4)
    ep = T.Epilogue()
    ep.kind, ep.ldo, ep.out = T.EPI_STORE_F32, N, y.ptr

    def run(i):
        t, s = W[i % copies]
        T.check(L.ti_gemm_wq_a16(t.ptr, s.ptr, bits, x16.ptr, T.X_F16, K, None, 1e-5, 1, N, K, C.byref(ep), None))

    for i in range(copies):
        run(i)
    T.sync()
    reps = max(64, 8 * copies)
    T.check(L.ti_event_record(ev0, None))
    for i in range(reps):
        run(i)
    T.check(L.ti_event_record(ev1, None))
    ms = C.c_float()
    T.check(L.ti_event_elapsed_ms(ev0, ev1, C.byref(ms)))
    us = ms.value * 1e3 / reps
    grid = L.ti_gemm_grid(1, N, K)
    print(f"{name:13s} bits={bits} K={K:6d} N={N:6d} grid={grid:4d} {(tb + sb) / max(grid, 1) / 1024:7.1f} KiB/wg "
          f"{us:7.2f} us  {(tb + sb) / us / 1e3:7.1f} GB/s", flush=True)
    del W
