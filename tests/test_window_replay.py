"""The recent window's replay of a run's lookup hits on the host (xc_memcache.cpp): the whole-run
replay with chunks simulated ahead on helper threads (xc__mem_hits_run) leaves the window the
reference's lookups build (xcodec/xcodec_cache.h:130-147: a map hit not in the 64-entry window is
remembered in the next slot, round robin), checked against a plain FIFO model and against the
buffer-by-buffer replay.  Host code only: no GPU."""
import ctypes as C

import numpy as np
import pytest

from wanproxy_amd.xcodec import load_library

STRIDE = 17  # COLL_CAP + 1 (the runtime's packing; any stride works for the layout)


def _lib():
    lib = load_library()
    lib.xc__mem_new.restype = C.c_void_p
    lib.xc__mem_new.argtypes = [C.c_void_p, C.c_void_p]
    lib.xc__mem_free.argtypes = [C.c_void_p]
    lib.xc__mem_hits.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int]
    lib.xc__mem_hits_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32]
    lib.xc__mem_window.argtypes = [C.c_void_p, C.c_void_p]
    return lib


def _pack(runs):
    """Buffers' hit lists -> (h, tok_base) in the runtime's layout."""
    tok_base = np.zeros(len(runs) + 1, np.uint32)
    for b, r in enumerate(runs):
        tok_base[b + 1] = tok_base[b] + len(r)
    h = np.zeros(int(tok_base[-1]) + len(runs) * STRIDE, np.uint64)
    for b, r in enumerate(runs):
        o = int(tok_base[b]) + b * STRIDE
        h[o] = len(r)
        h[o + 1:o + 1 + len(r)] = r
    return h, tok_base


def _fifo(stream, win=None):
    """The reference's window after the stream: insert a hash not present at the next slot."""
    w = list(win) if win is not None else []
    for x in stream:
        if x not in w:
            w.append(x)
            if len(w) > 64:
                w.pop(0)
    return w


def _window(lib, m):
    out = np.zeros(64, np.uint64)
    lib.xc__mem_window(m, out.ctypes.data)
    return [int(v) for v in out if v]


@pytest.mark.parametrize("pool,nb,per", [(80, 3000, 16), (8192, 4096, 16), (1 << 40, 2048, 9),
                                         (300, 5000, 3), (65, 2000, 40)])
def test_whole_run_replay_equals_the_fifo(pool, nb, per):
    lib = _lib()
    rng = np.random.default_rng(pool ^ nb)
    keys = rng.integers(1, 2**63, size=min(pool, 1 << 20), dtype=np.uint64)
    runs = []
    for b in range(nb):
        k = int(rng.integers(0, 2 * per + 1))
        if pool < (1 << 20):
            runs.append(keys[rng.integers(0, pool, k)])
        else:
            runs.append(rng.integers(1, 2**63, size=k, dtype=np.uint64))
    m_run, m_seq = lib.xc__mem_new(None, None), lib.xc__mem_new(None, None)
    try:
        # a first run replayed buffer by buffer leaves a full window behind (the next run's true start)
        pre = [keys[rng.integers(0, min(pool, len(keys)), 100)] for _ in range(4)]
        for r in pre:
            for m in (m_run, m_seq):
                lib.xc__mem_hits(m, np.ascontiguousarray(r).ctypes.data, len(r), 1)
        h, tb = _pack(runs)
        lib.xc__mem_hits_run(m_run, h.ctypes.data, tb.ctypes.data, STRIDE, nb)
        for r in runs:
            r = np.ascontiguousarray(r, np.uint64)
            lib.xc__mem_hits(m_seq, r.ctypes.data, len(r), 1)
        want = _fifo(np.concatenate(runs), _fifo(np.concatenate(pre)))
        assert _window(lib, m_seq) == [int(x) for x in want]
        assert _window(lib, m_run) == [int(x) for x in want]
    finally:
        lib.xc__mem_free(m_run)
        lib.xc__mem_free(m_seq)


def test_whole_run_replay_with_hash_zero_and_repeats():
    """Hash 0 (the unused slots' hash) in a chunk, and a chunk that keeps hitting the 64 hashes the
    window holds (no insertion for long stretches): the exact replay decides every hit."""
    lib = _lib()
    rng = np.random.default_rng(7)
    keys = rng.integers(1, 2**63, size=64, dtype=np.uint64)
    runs = []
    for b in range(3000):
        if 1500 <= b < 1600:
            runs.append(keys[rng.integers(0, 64, 8)])         # the window's own hashes only
        elif b == 2100:
            runs.append(np.array([0, 5, 0], np.uint64))
        else:
            runs.append(rng.integers(1, 2**63, size=int(rng.integers(0, 20)), dtype=np.uint64))
    m_run, m_seq = lib.xc__mem_new(None, None), lib.xc__mem_new(None, None)
    try:
        h, tb = _pack(runs)
        lib.xc__mem_hits_run(m_run, h.ctypes.data, tb.ctypes.data, STRIDE, len(runs))
        for r in runs:
            r = np.ascontiguousarray(r, np.uint64)
            lib.xc__mem_hits(m_seq, r.ctypes.data, len(r), 1)
        out_run, out_seq = np.zeros(64, np.uint64), np.zeros(64, np.uint64)
        lib.xc__mem_window(m_run, out_run.ctypes.data)
        lib.xc__mem_window(m_seq, out_seq.ctypes.data)
        assert np.array_equal(out_run, out_seq)
    finally:
        lib.xc__mem_free(m_run)
        lib.xc__mem_free(m_seq)


@pytest.mark.parametrize("threads", ["0", "1", "3"])
def test_replay_threads_knob(threads):
    """XC_REPLAY_THREADS (the helper threads of the whole-run replay, read once per process): with
    none, one or three helpers the window still equals the FIFO model's (a fresh process each)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, XC_REPLAY_THREADS=threads)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(root, "tests", "test_window_replay.py"), "-k", "fifo or zero_and_repeats"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
