"""Full-size parity: the gfx950 engine on the exact bench workloads against the oracle's runs.

tests/golden/fullsize_<config>.json holds the oracle's (and, for C1/C2, also the seeded reference
CLI's) results on the workloads bench.py times — klsh-synth v1 counts, the mode-C conversion, the
init pass (app/kmerLSH.cc:323), then the main Cluster() loop (app/kmerLSH.cc:490,
function/cluster.cc:181-340).  C1, C2 and C4 (100M x 32) are pinned over their whole loop (10,
500 and 100 iterations; the C4 fixture took the oracle 31 min on 6 threads); C5 (10M x 512) over
the first 100 of its 500 iterations (33 min), and its full loop is checked through
size-independent properties: N_t non-increasing, the prefix of the full run equal to the pinned
prefix, member lists partitioning the kept rows, and a bit-identical replay.

Bar: bit-exact (N_t trace, rng counter, md5 of the fp32 row bits, member offsets and ids).
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
            if "reference" in fx:  # the reference CLI agreed with the oracle on these files
                assert fx["reference"]["agrees"]
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
