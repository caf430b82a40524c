"""Full-size parity fixtures: the oracle run on the exact bench workloads (C1, C2, C4, C5).

TEST INFRASTRUCTURE (run in the build container, never on the GPU box).  For every config of
bench.py the workload is rebuilt exactly as bench.py's prepare() builds it — klsh-synth v1 counts
(the product's host generator, kmerlsh_amd/csrc/klsh_synth.cpp), the mode-C conversion
(io/ioMatrix.cc:353-408), the init pass (one iteration at 0.95, bucket threshold 1e5;
app/kmerLSH.cc:323) — and then the main Cluster() loop (app/kmerLSH.cc:490,
function/cluster.cc:181-340) runs in the oracle (oracle/klsh_oracle.c, pinned bit-for-bit against
the reference's own outputs by tests/test_oracle_golden.py).  Every config is pinned over its
whole loop (round 6: C5's 500 iterations too; a config can still be pinned on a prefix, the first
`run` iterations of the `iters`-iteration threshold schedule, klsh_oracle_cluster_prefix).

Stored per config (tests/golden/fullsize_<config>.json): the init-pass trace and survivors, the main
loop's N_t trace, the rng counter, Σ N_t, the final count, and md5s of the result in canonical
order (fp32 row bits, uint64 member offsets, uint64 member ids).  tests/test_gpu_fullsize.py
compares the gfx950 engine against these, bit-exact.

    python tests/golden/make_fullsize.py [c1 c2 c4 c5] [--threads 8] [--reference]

With --reference (full loops only) the seeded reference CLI itself also runs mode C at -T 1 on the
same count files; its N_t trace and clustering_result.txt(.clust) md5s must equal the oracle's.
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import klsh_oracle  # noqa: E402
from kmerlsh_amd import _native  # noqa: E402
from kmerlsh_amd.io import save_binary, save_result, v_kmers_from_coverage, write_count_files  # noqa: E402

REF_CLI = os.path.join(ROOT, "oracle", "_ref", "kmerLSH_seeded")

def out_path(name: str) -> str:
    return os.path.join(HERE, f"fullsize_{name}.json")

# name: (kmers, samples, synth seed, -I, iterations pinned, min_similarity); the same workloads as
# bench.py's CONFIGS (seeds per SURVEY.md §8(d))
FULLSIZE = {
    "c1": (100_000, 8, 1, 10, 10, 0.80),
    "c2": (10_000_000, 64, 11, 500, 500, 0.80),
    "c4": (100_000_000, 32, 13, 100, 100, 0.80),
    "c5": (10_000_000, 512, 17, 500, 500, 0.80),
}
SEED_BASE = 12345
INIT_BTHR = 100_000     # app/kmerLSH.cc:285,323 (batch_thresh / 1000)
MAIN_BTHR = 1_000_000   # app/kmerLSH.cc:440,490


def md5(a: np.ndarray) -> str:
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()


def file_md5(path: str) -> str:
    h = hashlib.md5()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 24), b""):
            h.update(chunk)
    return h.hexdigest()


def written_md5(out, off, ids) -> dict:
    """md5 of clustering_result.txt / .clust as the reference CLI writes them (clusters with more
    than 5 members, io/ioMatrix.cc:265-294,322-351, app/kmerLSH.cc:498-499)."""
    with tempfile.TemporaryDirectory() as tmp:
        f = os.path.join(tmp, "clustering_result.txt")
        save_result(f + ".clust", off, ids)
        save_binary(f, out, off)
        return {"clustering_result.txt": file_md5(f),
                "clustering_result.txt.clust": file_md5(f + ".clust")}


def run_reference(name: str, counts: np.ndarray, cov: np.ndarray) -> dict:
    """The seeded reference CLI itself (oracle/_ref/kmerLSH_seeded) in mode C at
    -T 1 on the same count files: its outputs and N_t trace pin the oracle at full size."""
    n, d, seed, iters, run_iters, min_sim = FULLSIZE[name]
    assert run_iters == iters
    t0 = time.time()
    with tempfile.TemporaryDirectory() as wd:
        write_count_files(wd, counts, cov)
        os.makedirs(os.path.join(wd, "tmp"))
        env = dict(os.environ, OMP_THREAD_LIMIT="1", OMP_NUM_THREADS="1", KLSH_SEED=str(SEED_BASE))
        so = subprocess.run([REF_CLI, "-a", "a.txt", "-b", "b.txt", "-o", "A", "-p", "B",
                             "-I", str(iters), "-N", "%.2f" % min_sim, "-K", "23", "-T", "1",
                             "-M", "C", "--only", "--verbose"], env=env, cwd=wd, check=True,
                            capture_output=True, text=True).stdout
        sizes = [int(v) for v in re.findall(r"Size of profilings\D*(\d+)", so)]
        # the main loop's own timer (function/cluster.cc:335-338: the last "hash+cluster takes"
        # line is the main Cluster() call, app/kmerLSH.cc:490)
        loops = [float(v) for v in re.findall(r"hash\+cluster takes \(secs\): ([0-9.eE+-]+)", so)]
        md5 = {fn: file_md5(os.path.join(wd, fn))
               for fn in ("clustering_result.txt", "clustering_result.txt.clust")}
    return {"trace": sizes[-iters:], "init_trace": sizes[:-iters], "md5": md5,
            "seconds": round(time.time() - t0, 1),
            "main_loop_seconds": loops[-1] if loops else None,
            "host": "build container (8-core Xeon), OMP_THREAD_LIMIT=1 -T 1"}


def run(name: str, threads: int, reference: bool = False) -> dict:
    n, d, seed, iters, run_iters, min_sim = FULLSIZE[name]
    L = klsh_oracle.lib()
    L.klsh_oracle_cluster_prefix.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int,
                                             ctypes.POINTER(klsh_oracle.Rng), ctypes.c_void_p,
                                             ctypes.c_int]
    L.klsh_oracle_cluster_prefix.restype = ctypes.c_int
    p = klsh_oracle._p
    t0 = time.time()
    counts, cov = _native.synth_counts(n, d, seed=seed)
    v_kmers = v_kmers_from_coverage(cov, n)
    rows, _ = klsh_oracle.convert(counts, v_kmers)
    if not reference:
        del counts
    kept = rows.shape[0]
    st = L.klsh_oracle_create(p(rows), kept, d, None, None)
    del rows
    try:
        rng = klsh_oracle.Rng(SEED_BASE, 0)
        itrace = np.zeros(1, dtype=np.uint64)
        L.klsh_oracle_cluster(st, ctypes.c_float(0.80), 1, INIT_BTHR, ctypes.byref(rng), p(itrace),
                              threads)
        n_init = L.klsh_oracle_count(st)
        counter_init = rng.counter
        print(f"[{name}] kept {kept}, init -> {n_init} ({time.time() - t0:.0f}s)", flush=True)
        trace = np.zeros(iters, dtype=np.uint64)
        ran = L.klsh_oracle_cluster_prefix(st, ctypes.c_float(min_sim), iters, run_iters,
                                           MAIN_BTHR, ctypes.byref(rng), p(trace), threads)
        assert ran == run_iters
        c = L.klsh_oracle_count(st)
        m = L.klsh_oracle_members(st)
        out = np.zeros((c, d), dtype=np.float32)
        off = np.zeros(c + 1, dtype=np.uint64)
        ids = np.zeros(m, dtype=np.uint64)
        L.klsh_oracle_result(st, p(out), p(off), p(ids))
    finally:
        L.klsh_oracle_destroy(st)
    rec = {
        "kmers": n, "samples": d, "synth_seed": seed, "seed_base": SEED_BASE,
        "iterations": iters, "run_iterations": run_iters, "min_similarity": min_sim,
        "init_bucket_threshold": INIT_BTHR, "main_bucket_threshold": MAIN_BTHR,
        "kept": int(kept), "init_trace": [int(v) for v in itrace], "n_init": int(n_init),
        "counter_init": int(counter_init),
        "trace": [int(v) for v in trace[:run_iters]], "sum_trace": int(trace[:run_iters].sum()),
        "counter": int(rng.counter), "n_final": int(c), "n_members": int(off[-1]),
        "md5_rows": md5(out), "md5_offsets": md5(off), "md5_ids": md5(ids[: int(off[-1])]),
        "oracle_seconds": round(time.time() - t0, 1), "oracle_threads": threads,
    }
    print(f"[{name}] final {c} clusters, sum N_t {rec['sum_trace']}, "
          f"{rec['oracle_seconds']}s", flush=True)
    if run_iters == iters:
        rec["written_md5"] = written_md5(out, off, ids[: int(off[-1])])
    if reference:
        ref = run_reference(name, counts, cov)
        rec["reference"] = ref
        rec["reference"]["agrees"] = (ref["md5"] == rec["written_md5"] and
                                      ref["trace"] == rec["trace"] and
                                      ref["init_trace"] == rec["init_trace"])
        print(f"[{name}] reference CLI ({ref['seconds']}s): agrees = {ref['agrees']}", flush=True)
        assert ref["agrees"], ref
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=list(FULLSIZE))
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--reference", action="store_true",
                    help="also run the seeded reference CLI at -T 1 (full loops only; C2 ~1 h)")
    args = ap.parse_args()
    for name in args.configs:
        rec = run(name, args.threads, args.reference)
        with open(out_path(name), "w") as f:
            json.dump(rec, f, indent=1, sort_keys=True)
            f.write("\n")


if __name__ == "__main__":
    main()
