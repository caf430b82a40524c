"""Minimal C2 loop for profiling any engine build (KLSH_LIB=...): synth -> convert -> init pass ->
one 500-iteration main loop.  No statistics are interpreted (older builds have other layouts).
    python tools/run_c2.py [iterations]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kmerlsh_amd import _native  # noqa: E402
from kmerlsh_amd.io import v_kmers_from_coverage  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 500
n, d = 10_000_000, 64
counts, cov = _native.synth_counts(n, d, seed=11)
eng = _native.Engine(0)
eng.load_counts(counts, v_kmers_from_coverage(cov, n))
del counts
_, c0, _ = eng.cluster(0.80, 1, 100_000, 12345, 0)
t0 = time.perf_counter()
trace, c1, _ = eng.cluster(0.80, iters, 1_000_000, 12345, c0)
print(f"loop {1e3 * (time.perf_counter() - t0):.1f} ms, final {int(trace[-1])} rows", flush=True)
