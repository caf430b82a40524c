"""Full-size parity: the gfx950 engine on the exact bench workloads against the oracle's runs.

tests/golden/fullsize_<config>.json holds the oracle's results on the workloads bench.py times —
klsh-synth v1 counts, the mode-C conversion, the init pass (app/kmerLSH.cc:323), then the main
Cluster() loop (app/kmerLSH.cc:490, function/cluster.cc:181-340) — and, for C1 and C2, the seeded
reference CLI's own run on the same count files (-T 1; tests/golden/make_fullsize.py --reference:
its N_t trace and both output files' md5s equal the oracle's, `reference.agrees`).  All four are
pinned over their whole loop: C1 (10 iterations), C2 (500; the reference CLI took 37 min), C4
(100M x 32, 100; the oracle 31 min on 6 threads) and C5 (10M x 512, 500; the oracle 33 min on 6
threads, round 6 — rounds 3-5 pinned its first 100 iterations).  A fixture pinned on a prefix
only is checked over its whole loop through size-independent properties (N_t non-increasing,
member lists partitioning the kept rows, a bit-identical replay).

Bar: bit-exact (N_t trace, rng counter, md5 of the fp32 row bits, member offsets and ids, and of
clustering_result.txt / .clust as written — for C1 and C2 the reference CLI's own files).
"""
import glob
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FIXTURES = sorted(os.path.basename(p)[len("fullsize_"):-len(".json")]
                  for p in glob.glob(os.path.join(GOLDEN, "fullsize_*.json")))


def fixture(name):
    with open(os.path.join(GOLDEN, f"fullsize_{name}.json")) as f:
        return json.load(f)


def md5(a):
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()


def prepare(eng, fx):
    """bench.py's prepare(): synth -> GPU mode-C conversion -> init pass; then a snapshot."""
    from kmerlsh_amd import _native
    from kmerlsh_amd.io import v_kmers_from_coverage

    n, d = fx["kmers"], fx["samples"]
    counts, cov = _native.synth_counts(n, d, seed=fx["synth_seed"])
    eng.load_counts(counts, v_kmers_from_coverage(cov, n))
    del counts
    kept, _ = eng.count()
    assert kept == fx["kept"]
    itrace, counter, _ = eng.cluster(0.80, 1, fx["init_bucket_threshold"], fx["seed_base"], 0)
    assert itrace.tolist() == fx["init_trace"]
    assert counter == fx["counter_init"]
    assert eng.count()[0] == fx["n_init"]
    eng.snapshot()


def main_loop(eng, fx, stop_after=0):
    eng.restore()
    eng.set_option("stop_after", stop_after)
    try:
        trace, counter, st = eng.cluster(fx["min_similarity"], fx["iterations"],
                                         fx["main_bucket_threshold"], fx["seed_base"],
                                         fx["counter_init"])
    finally:
        eng.set_option("stop_after", 0)
    rows, off, ids = eng.result()
    return trace, counter, rows, off, ids


def written_md5(rows, off, ids):
    """md5 of clustering_result.txt / .clust as kmerLSH -M C writes them (io/ioMatrix.cc:265-351,
    clusters with more than 5 members, app/kmerLSH.cc:498-499)."""
    import tempfile

    from kmerlsh_amd.io import save_binary, save_result

    with tempfile.TemporaryDirectory() as tmp:
        f = os.path.join(tmp, "clustering_result.txt")
        save_result(f + ".clust", off, ids)
        save_binary(f, rows, off)
        out = {}
        for fn in ("clustering_result.txt", "clustering_result.txt.clust"):
            with open(os.path.join(tmp, fn), "rb") as fh:
                out[fn] = hashlib.md5(fh.read()).hexdigest()
        return out


def assert_pinned(fx, trace, counter, rows, off, ids):
    assert trace.tolist() == fx["trace"]
    assert counter == fx["counter"]
    assert rows.shape[0] == fx["n_final"] and int(off[-1]) == fx["n_members"]
    assert md5(off) == fx["md5_offsets"]
    assert md5(ids) == fx["md5_ids"]
    assert md5(rows) == fx["md5_rows"]


@pytest.mark.parametrize("name", FIXTURES)
def test_fullsize_matches_oracle(name):
    from kmerlsh_amd import _native

    fx = fixture(name)
    with _native.Engine(0) as eng:
        prepare(eng, fx)
        full = fx["run_iterations"] == fx["iterations"]
        pinned = main_loop(eng, fx, 0 if full else fx["run_iterations"])
        assert_pinned(fx, *pinned)
        if full:
            if "written_md5" in fx:  # the files the CLI writes from this result (>5 members)
                assert written_md5(*pinned[2:]) == fx["written_md5"]
            if "reference" in fx:  # the reference CLI wrote these same files
                assert fx["reference"]["agrees"]
                assert fx["reference"]["md5"] == fx["written_md5"]
            return
        # the whole loop at size: properties (and a bit-identical replay)
        trace, counter, rows, off, ids = main_loop(eng, fx)
        assert len(trace) == fx["iterations"]
        assert trace[: fx["run_iterations"]].tolist() == fx["trace"]
        assert np.all(np.diff(trace.astype(np.int64)) <= 0)
        assert rows.shape[0] <= int(trace[-1])
        assert int(off[-1]) == fx["kept"]
        assert np.all(np.diff(off.astype(np.int64)) >= 1)
        seen = np.zeros(fx["kept"], dtype=np.bool_)
        seen[ids.astype(np.int64)] = True
        assert seen.all()  # every kept row is in exactly one cluster (sizes sum to kept)
        assert np.isfinite(rows).all()
        again = main_loop(eng, fx)
        assert again[0].tolist() == trace.tolist() and again[1] == counter
        assert md5(again[2]) == md5(rows) and md5(again[3]) == md5(off)
        assert md5(again[4]) == md5(ids)
