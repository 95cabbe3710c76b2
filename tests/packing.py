"""Test helpers: a numpy reader of the packed tile format (include/ti_hip.h) so packed weights
can be compared with the oracle's quantizer, and reference-layout dequantization."""
from __future__ import annotations

import numpy as np


def unpack_tiles(tiles: np.ndarray, scales: np.ndarray, bits: int, K: int, N: int):
    """-> (q [N][K] int8 or fp16 weights [N][K], scales [N][K/128] uint16 or None)."""
    KT, NT = K // 128, N // 16
    chunks = bits // 4
    t = np.asarray(tiles, np.uint8).reshape(NT, KT, chunks, 64, 16)
    lane = np.arange(64)
    r, kq = lane & 15, lane >> 4
    if bits == 16:
        h = t.view(np.uint16).reshape(NT, KT, chunks, 64, 8)
        out = np.zeros((N, K), np.uint16)
        for c in range(chunks):
            for e in range(8):
                k = kq * 32 + c * 8 + e        # per lane
                for nt in range(NT):
                    out[nt * 16 + r[:, None], (np.arange(KT)[None, :] * 128 + k[:, None])] = h[nt, :, c, :, e].T
        return out.view(np.float16), None
    q = np.zeros((N, K), np.int8)
    if bits == 4:
        w = t.view(np.uint32).reshape(NT, KT, 64, 4)
        for s4 in range(4):
            for e in range(8):
                p = e >> 1
                shift = (16 + 4 * p) if (e & 1) else (4 * p)
                nib = ((w[:, :, :, s4] >> shift) & 0xF).astype(np.int16) - 8    # [NT][KT][64]
                k = kq * 32 + s4 * 8 + e
                for nt in range(NT):
                    q[nt * 16 + r[:, None], np.arange(KT)[None, :] * 128 + k[:, None]] = nib[nt].T
    else:
        b = t.view(np.int8).reshape(NT, KT, 2, 64, 16)
        for c in range(2):
            for j in range(16):
                k = kq * 32 + c * 16 + j
                for nt in range(NT):
                    q[nt * 16 + r[:, None], np.arange(KT)[None, :] * 128 + k[:, None]] = b[nt, :, c, :, j].T
    s = np.asarray(scales, np.uint16).reshape(NT, KT, 16).transpose(0, 2, 1).reshape(N, KT)
    return q, s


def dequant_ref_layout(q: np.ndarray, s: np.ndarray) -> np.ndarray:
    """q [N][K], s [N][K/128] fp16 bits -> W [K][N] fp32 = float(q) * float(s)."""
    N, K = q.shape
    sf = s.view(np.float16).astype(np.float32)
    w = q.astype(np.float32) * np.repeat(sf, 128, axis=1)
    return np.ascontiguousarray(w.T)
