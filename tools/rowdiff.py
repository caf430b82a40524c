"""Diagnostics (GPU box): the engine and the oracle on one klsh-synth workload, row by row.

Builds the workload as bench.py / tests/golden/make_fullsize.py do (synth counts, mode-C
conversion, init pass), runs the first `--run` iterations of the `--iters`-iteration schedule on
both, and prints the result rows whose fp32 bits differ (with their member counts), plus the first
iteration whose N_t differs.  Test infrastructure: imports the oracle.

    python tools/rowdiff.py --n 1000000 --d 512 --seed 17 --iters 500 --run 20
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import klsh_oracle  # noqa: E402
from kmerlsh_amd import _native  # noqa: E402
from kmerlsh_amd.io import v_kmers_from_coverage  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--d", type=int, default=512)
ap.add_argument("--seed", type=int, default=17)
ap.add_argument("--iters", type=int, default=500)
ap.add_argument("--run", type=int, default=20)
ap.add_argument("--threads", type=int, default=16)
a = ap.parse_args()
SEED_BASE = 12345

counts, cov = _native.synth_counts(a.n, a.d, seed=a.seed)
vk = v_kmers_from_coverage(cov, a.n)
t0 = time.time()
with _native.Engine(0) as eng:
    eng.load_counts(counts, vk)
    _, c0, _ = eng.cluster(0.80, 1, 100_000, SEED_BASE, 0)
    eng.set_option("stop_after", a.run)
    g_trace, g_counter, _ = eng.cluster(0.80, a.iters, 1_000_000, SEED_BASE, c0)
    g_rows, g_off, g_ids = eng.result()
print(f"gpu {time.time() - t0:.1f}s: {g_rows.shape[0]} rows", flush=True)

t0 = time.time()
L = klsh_oracle.lib()
L.klsh_oracle_cluster_prefix.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(klsh_oracle.Rng),
                                         ctypes.c_void_p, ctypes.c_int]
L.klsh_oracle_cluster_prefix.restype = ctypes.c_int
p = klsh_oracle._p
rows, _ = klsh_oracle.convert(counts, vk)
st = L.klsh_oracle_create(p(rows), rows.shape[0], a.d, None, None)
rng = klsh_oracle.Rng(SEED_BASE, 0)
it = np.zeros(1, dtype=np.uint64)
L.klsh_oracle_cluster(st, ctypes.c_float(0.80), 1, 100_000, ctypes.byref(rng), p(it), a.threads)
assert rng.counter == c0, (rng.counter, c0)
trace = np.zeros(a.iters, dtype=np.uint64)
L.klsh_oracle_cluster_prefix(st, ctypes.c_float(0.80), a.iters, a.run, 1_000_000, ctypes.byref(rng),
                             p(trace), a.threads)
c = L.klsh_oracle_count(st)
m = L.klsh_oracle_members(st)
o_rows = np.zeros((c, a.d), dtype=np.float32)
o_off = np.zeros(c + 1, dtype=np.uint64)
o_ids = np.zeros(m, dtype=np.uint64)
L.klsh_oracle_result(st, p(o_rows), p(o_off), p(o_ids))
L.klsh_oracle_destroy(st)
print(f"oracle {time.time() - t0:.1f}s: {c} rows", flush=True)

o_trace = trace[: a.run]
if g_trace[: a.run].tolist() != o_trace.tolist():
    k = next(i for i in range(a.run) if g_trace[i] != o_trace[i])
    print(f"TRACE differs first at iteration {k}: gpu {g_trace[k]} oracle {o_trace[k]}")
print("counter", g_counter, rng.counter, "offsets equal", np.array_equal(g_off, o_off),
      "ids equal", np.array_equal(g_ids, o_ids[: int(o_off[-1])]))
if g_rows.shape == o_rows.shape:
    gb, ob = g_rows.view(np.uint32), o_rows.view(np.uint32)
    bad = np.nonzero((gb != ob).any(axis=1))[0]
    print(f"{bad.size} rows differ")
    sizes = np.diff(o_off.astype(np.int64))
    for r in bad[:20]:
        cols = np.nonzero(gb[r] != ob[r])[0]
        ulp = np.abs(gb[r, cols].astype(np.int64) - ob[r, cols].astype(np.int64))
        print(f"  row {r}: members {sizes[r]}, {cols.size} columns differ (first {cols[:6].tolist()}),"
              f" max ulp {ulp.max()}, gpu {g_rows[r, cols[0]]!r} oracle {o_rows[r, cols[0]]!r}")
    if bad.size:
        print("member-count histogram of differing rows:",
              np.unique(sizes[bad], return_counts=True))
