"""One tile-GEMM shape timed in a loop (for rocprofv3 --pmc passes): 7B QKV at 512 rows by default.
    python tools/tile_one.py [M N K reps]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

M, N, K, reps = (int(v) for v in (sys.argv[1:5] if len(sys.argv) >= 5 else (512, 12288, 4096, 20)))
T.init(0)
L = T.lib()
tb, sb = L.ti_wpack_tile_bytes(4, K, N), L.ti_wpack_scale_bytes(4, K, N)
tiles, scales = T.DeviceBuffer(tb), T.DeviceBuffer(sb)
T.check(L.ti_wsynth_device(1, 7, K, N, N, 4, 0, 0, tiles.ptr, scales.ptr, None))
x = T.DeviceBuffer.from_array(np.random.RandomState(0).standard_normal((M, K)).astype(np.float16))
y = T.DeviceBuffer(M * N * 4)
ep = T.Epilogue()
ep.kind, ep.ldo, ep.out = T.EPI_STORE_F32, N, y.ptr
for _ in range(reps):
    T.check(L.ti_gemm_wq_a16(tiles.ptr, scales.ptr, 4, x.ptr, T.X_F16, K, None, 1e-5, M, N, K, C.byref(ep), None))
T.sync()
print("ok", M, N, K, reps)
