"""Engines driven from other host threads and (when the box has them) other devices
(one engine per GPU).  Every ti_engine_* entry binds the
engine's device for the call and restores the caller's (engine.cpp DeviceScope): a call from a
thread whose current device differs -- or that never selected one -- allocates, captures and
launches on the engine's device and gives the same results as on the creating thread."""
from __future__ import annotations

import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CFG = (1024, 512, 2, 8, 2, 64, 768)   # vocab, hidden, layers, heads, kv_heads, head_dim, inter


def _engine(ti, device=0, max_batch=4):
    v, h, l, nh, nkv, hd, inter = CFG
    e = ti.Engine(v, h, l, nh, nkv, hd, inter, bits=4, max_seq=256, max_batch=max_batch, device=device)
    e.synth(77, 0.1)
    return e


def _work(e):
    g = np.asarray(e.generate([[1, 2, 3], [9]], 8))
    s = [np.asarray(t) for t in e.serve([[4, 5], [6], [7, 8, 9], [10]], 6, chunk=3)]
    b = e.beam_search([1, 2, 3], 5, 3)
    return g, s, b


def _in_thread(fn, *args):
    out, err = {}, {}

    def run():
        try:
            out["v"] = fn(*args)
        except BaseException as ex:   # re-raised on the calling thread
            err["e"] = ex

    t = threading.Thread(target=run)
    t.start()
    t.join(300)
    assert not t.is_alive(), "worker thread hung"
    if err:
        raise err["e"]
    return out["v"]


def _same(a, b):
    assert np.array_equal(a[0], b[0])
    assert len(a[1]) == len(b[1]) and all(np.array_equal(x, y) for x, y in zip(a[1], b[1]))
    assert [(r[0], r[1]) for r in a[2]] == [(r[0], r[1]) for r in b[2]]


def test_engine_created_here_used_from_another_thread(ti):
    ref_e = _engine(ti)
    ref = _work(ref_e)
    ref_e.close()
    e = _engine(ti)                     # created (and its weights synthesised) on this thread
    got = _in_thread(_work, e)          # generate, serve and beam search from a worker thread
    _same(got, ref)
    got2 = _work(e)                     # and back on the creating thread
    _same(got2, ref)
    e.close()


def test_engine_created_in_another_thread(ti):
    ref_e = _engine(ti)
    ref = _work(ref_e)
    ref_e.close()
    e = _in_thread(_engine, ti)
    _same(_work(e), ref)
    _in_thread(e.close)


@pytest.mark.skipif("not __import__('turboinfer_amd').device_count() > 1")
def test_two_devices_two_threads(ti):
    """One engine per device, each driven from its own thread concurrently, plus a call on the
    second device's engine from a thread whose current device is the first."""
    ref_e = _engine(ti, 0)
    ref = _work(ref_e)
    ref_e.close()
    engines = [_engine(ti, d) for d in (0, 1)]
    results = [None, None]

    def run(i):
        results[i] = _work(engines[i])

    ts = [threading.Thread(target=run, args=(i,)) for i in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    for r in results:
        _same(r, ref)
    _same(_work(engines[1]), ref)
    for e in engines:
        e.close()
