"""TEST INFRASTRUCTURE ONLY — ctypes binding of the plain-C oracle (oracle/libklsh_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this, and only
as the checker / the timed CPU baseline.  The product (kmerlsh_amd/) never imports it.
Parity status: PINNED (see klsh_oracle.h).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libklsh_oracle.so")
CLI = os.path.join(HERE, "klsh_oracle")
REF_HARNESS = os.path.join(HERE, "_ref", "ref_harness")
REF_CLI = os.path.join(HERE, "_ref", "kmerLSH_seeded")

_lib = None
_P = ctypes.c_void_p


class Rng(ctypes.Structure):
    _fields_ = [("base", ctypes.c_uint32), ("counter", ctypes.c_uint64)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.klsh_oracle_hyperplane.argtypes = [ctypes.c_uint32, ctypes.c_int, _P]
        L.klsh_oracle_table.argtypes = [ctypes.POINTER(Rng), ctypes.c_int, ctypes.c_int, _P]
        L.klsh_oracle_key.argtypes = [_P, ctypes.c_int, _P, ctypes.c_int]
        L.klsh_oracle_key.restype = ctypes.c_uint32
        L.klsh_oracle_cosine.argtypes = [_P, _P, ctypes.c_int]
        L.klsh_oracle_cosine.restype = ctypes.c_float
        L.klsh_oracle_consensus.argtypes = [_P, ctypes.c_uint32, _P, ctypes.c_uint32,
                                            ctypes.c_int, _P]
        L.klsh_oracle_create.argtypes = [_P, ctypes.c_uint64, ctypes.c_int, _P, _P]
        L.klsh_oracle_create.restype = _P
        L.klsh_oracle_destroy.argtypes = [_P]
        L.klsh_oracle_count.argtypes = [_P]
        L.klsh_oracle_count.restype = ctypes.c_uint64
        L.klsh_oracle_members.argtypes = [_P]
        L.klsh_oracle_members.restype = ctypes.c_uint64
        L.klsh_oracle_cluster.argtypes = [_P, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(Rng), _P, ctypes.c_int]
        L.klsh_oracle_cluster.restype = ctypes.c_int
        L.klsh_oracle_result.argtypes = [_P, _P, _P, _P]
        L.klsh_oracle_pcluster.argtypes = [_P, ctypes.c_float]
        L.klsh_oracle_pcluster.restype = ctypes.c_uint64
        L.klsh_oracle_convert.argtypes = [_P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_int, _P, _P, _P]
        L.klsh_oracle_convert.restype = ctypes.c_uint64
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def table(seed: int, counter: int, h: int, d: int) -> tuple[np.ndarray, int]:
    r = Rng(seed, counter)
    w = np.zeros((max(h, 0), d), dtype=np.float32)
    lib().klsh_oracle_table(ctypes.byref(r), h, d, _p(w))
    return w, r.counter


def keys(rows: np.ndarray, w: np.ndarray) -> np.ndarray:
    rows = np.ascontiguousarray(rows, np.float32)
    w = np.ascontiguousarray(w, np.float32)
    L = lib()
    d = rows.shape[1]
    out = np.zeros(rows.shape[0], dtype=np.uint32)
    for i in range(rows.shape[0]):
        out[i] = L.klsh_oracle_key(_p(rows[i]), d, _p(w), w.shape[0])
    return out


def cluster(rows: np.ndarray, min_sim: float, iters: int, bthr: int, seed: int = 12345,
            counter: int = 0, member_offsets=None, member_ids=None, threads: int = 0):
    """Cluster() at T=1 semantics -> (rows, offsets, ids, trace, counter)."""
    rows = np.ascontiguousarray(rows, np.float32)
    n, d = rows.shape
    mo = None if member_offsets is None else np.ascontiguousarray(member_offsets, np.uint64)
    mi = None if member_ids is None else np.ascontiguousarray(member_ids, np.uint64)
    L = lib()
    st = L.klsh_oracle_create(_p(rows), n, d, _p(mo), _p(mi))
    try:
        r = Rng(seed, counter)
        trace = np.zeros(max(iters, 1), dtype=np.uint64)
        ran = L.klsh_oracle_cluster(st, ctypes.c_float(min_sim), iters, bthr, ctypes.byref(r),
                                    _p(trace), threads)
        c = L.klsh_oracle_count(st)
        m = L.klsh_oracle_members(st)
        out = np.zeros((c, d), dtype=np.float32)
        off = np.zeros(c + 1, dtype=np.uint64)
        ids = np.zeros(m, dtype=np.uint64)
        L.klsh_oracle_result(st, _p(out), _p(off), _p(ids))
        return out, off, ids[: int(off[-1])], trace[:ran], r.counter
    finally:
        L.klsh_oracle_destroy(st)


def pcluster(rows: np.ndarray, thr: float, member_offsets=None, member_ids=None):
    """p_cluster over all rows as one bucket -> (rows, offsets, ids)."""
    rows = np.ascontiguousarray(rows, np.float32)
    n, d = rows.shape
    mo = None if member_offsets is None else np.ascontiguousarray(member_offsets, np.uint64)
    mi = None if member_ids is None else np.ascontiguousarray(member_ids, np.uint64)
    L = lib()
    st = L.klsh_oracle_create(_p(rows), n, d, _p(mo), _p(mi))
    try:
        L.klsh_oracle_pcluster(st, ctypes.c_float(thr))
        c = L.klsh_oracle_count(st)
        m = L.klsh_oracle_members(st)
        out = np.zeros((c, d), dtype=np.float32)
        off = np.zeros(c + 1, dtype=np.uint64)
        ids = np.zeros(m, dtype=np.uint64)
        L.klsh_oracle_result(st, _p(out), _p(off), _p(ids))
        return out, off, ids[: int(off[-1])]
    finally:
        L.klsh_oracle_destroy(st)


def convert(counts: np.ndarray, v_kmers: np.ndarray, batch_offset: int = 0,
            batch_size: int | None = None):
    counts = np.ascontiguousarray(counts, np.uint16)
    d, n_total = counts.shape
    if batch_size is None:
        batch_size = n_total - batch_offset
    vk = np.ascontiguousarray(v_kmers, np.float32)
    rows = np.zeros((batch_size, d), dtype=np.float32)
    ids = np.zeros(batch_size, dtype=np.uint64)
    kept = lib().klsh_oracle_convert(_p(counts), n_total, batch_offset, batch_size, d, _p(vk),
                                     _p(rows), _p(ids))
    return rows[:kept], ids[:kept]
