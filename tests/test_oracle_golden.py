"""The oracle (oracle/klsh_oracle.c, a plain-C restatement) against the reference's own outputs.

Every fixture in tests/golden/ was produced by the unmodified reference objects
(tests/golden/make_golden.py drives oracle/_ref/ref_harness and oracle/_ref/kmerLSH_seeded), so
these tests pin the oracle bit-for-bit before it is trusted as the checker of the GPU engine.
CPU only.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)
import kat_inputs  # noqa: E402

C = np.uint32(2654435761)


def test_rng_tables_match_reference(oracle):
    z = golden("rng_tables.npz")
    for name in z.files:
        seed, h, d = (int(p[1:]) for p in name.split("_"))
        w, counter = oracle.table(seed, 0, h, d)
        assert counter == h
        assert np.array_equal(w.view(np.uint32), z[name].view(np.uint32)), name


def test_rng_survey_kat(oracle):
    # SURVEY.md §8(c) RNG KAT: seed 12345, generateHashTable(3, 8), hyperplane 0.
    w, _ = oracle.table(12345, 0, 3, 8)
    assert [f"{v:08x}" for v in w[0].view(np.uint32)] == [
        "3f1857e5", "3d2b5a29", "3f4cea13", "bd934bad", "bf858348", "bec326d9", "bf441db4",
        "bfc9e9a4"]
    x = np.array([1, -2, 0.5, 3, -1, 0.25, 2, -0.75], dtype=np.float32)
    assert oracle.keys(x[None, :], w)[0] == 5
    w1, _ = oracle.table(1, 0, 3, 8)
    assert oracle.keys(x[None, :], w1)[0] == 3


def test_rng_counter_convention(oracle):
    # hyperplane k of stream `base` is the first hyperplane of stream base + k*2654435761
    base, k = 12345, 100
    w_a, _ = oracle.table(base, k, 4, 16)
    w_b, _ = oracle.table(int((np.uint64(base) + np.uint64(k) * np.uint64(C)) % (1 << 32)), 0, 4, 16)
    assert np.array_equal(w_a, w_b)


@pytest.mark.parametrize("name", ["keys_d8", "keys_d16", "keys_d64", "keys_d13", "keys_d512"])
def test_keys_match_reference(oracle, name):
    z = golden(name + ".npz")
    w, _ = oracle.table(int(z["seed"]), 0, int(z["h"]), z["rows"].shape[1])
    assert np.array_equal(oracle.keys(z["rows"], w), z["keys"])


@pytest.mark.parametrize("name", ["pcluster_small", "pcluster_large", "pcluster_generic",
                                  "pcluster_d8"])
def test_pcluster_matches_reference(oracle, name):
    z = golden(name + ".npz")
    rows, off, ids = oracle.pcluster(z["rows"], float(z["thr"]))
    assert np.array_equal(off, z["out_off"])
    assert np.array_equal(ids, z["out_ids"])
    assert np.array_equal(rows.view(np.uint32), z["out_rows"].view(np.uint32))


CLUSTER_CASES = ["cluster_d16", "cluster_d64", "cluster_d12", "cluster_d8_init", "cluster_nested",
                 "cluster_nested_small"]


@pytest.mark.parametrize("name", CLUSTER_CASES)
def test_cluster_matches_reference(oracle, name):
    z = golden(name + ".npz")
    rows, off, ids, trace, counter = oracle.cluster(
        z["rows"], float(z["min_sim"]), int(z["iters"]), int(z["bthr"]), int(z["seed"]))
    assert np.array_equal(trace, z["trace"])
    assert np.array_equal(off, z["out_off"])
    assert np.array_equal(ids, z["out_ids"])
    assert np.array_equal(rows.view(np.uint32), z["out_rows"].view(np.uint32))


def test_cluster_weighted_matches_reference(oracle):
    z = golden("cluster_weighted.npz")
    rows, off, ids, trace, _ = oracle.cluster(
        z["rows"], float(z["min_sim"]), int(z["iters"]), int(z["bthr"]), int(z["seed"]),
        member_offsets=z["in_off"], member_ids=z["in_ids"])
    assert np.array_equal(trace, z["trace"])
    assert np.array_equal(off, z["out_off"])
    assert np.array_equal(ids, z["out_ids"])
    assert np.array_equal(rows.view(np.uint32), z["out_rows"].view(np.uint32))


def test_cluster_thread_count_invariant(oracle):
    z = golden("cluster_d16.npz")
    a = oracle.cluster(z["rows"], 0.8, 10, 1000000, 12345, threads=1)
    b = oracle.cluster(z["rows"], 0.8, 10, 1000000, 12345, threads=4)
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x), np.asarray(y))


def test_convert_matches_reference(oracle):
    z = golden("convert.npz")
    rows, ids = oracle.convert(z["counts"], z["v_kmers"])
    assert np.array_equal(ids, z["out_ids"])
    assert np.array_equal(rows.view(np.uint32), z["out_rows"].view(np.uint32))


def test_empty_input_is_noop(oracle):
    # The reference aborts on an empty vector; the restatement is a no-op.
    rows, off, ids, trace, counter = oracle.cluster(np.zeros((0, 8), np.float32), 0.8, 3, 10)
    assert rows.shape == (0, 8) and list(trace) == [0, 0, 0] and counter == 0


def test_single_row(oracle):
    x = np.ones((1, 8), np.float32)
    rows, off, ids, trace, counter = oracle.cluster(x, 0.8, 4, 10)
    assert list(trace) == [1, 1, 1, 1] and counter == 0  # h = 0: no hyperplanes drawn
    assert np.array_equal(rows, x) and list(ids) == [0]


@pytest.mark.parametrize("kat", ["katF", "katG", "katN"])
def test_kat_end_to_end(oracle, kat, tmp_path):
    """Whole mode-C pipeline (transform, init pass, main loop, writers) of the restatement CLI
    against the seeded reference CLI's output md5s."""
    with open(os.path.join(GOLDEN, "kat_md5.json")) as f:
        ref = json.load(f)[kat]
    kat_inputs.write_kat(kat, str(tmp_path))
    out = subprocess.run([oracle.CLI, "-a", "a.txt", "-b", "b.txt", "-I", "10", "-T", "2", "-M", "C",
                          "--only", "--seed", "12345", "--verbose"], cwd=tmp_path, check=True,
                         capture_output=True, text=True).stdout
    for fn, md5 in ref["md5"].items():
        with open(tmp_path / fn, "rb") as f:
            assert hashlib.md5(f.read()).hexdigest() == md5, fn
    trace = [int(line.split(":")[1]) for line in out.splitlines() if line.startswith("Size of")]
    assert trace == ref["trace"]


def test_oracle_cli_recluster_branch(oracle, tmp_path):
    """The oracle CLI's multi-batch init and re-cluster passes (app/kmerLSH.cc:303-411) through the
    test-only KLSH_TEST_BATCH_THRESH override: every pass appears in the trace, the survivors shrink
    below the threshold before the main loop, and the run is deterministic."""
    kat_inputs.write_kat("katF", str(tmp_path))
    env = dict(os.environ, KLSH_TEST_BATCH_THRESH="3000")
    runs = []
    for _ in range(2):
        out = subprocess.run([oracle.CLI, "-a", "a.txt", "-b", "b.txt", "-I", "10", "-T", "2",
                              "-M", "C", "--only", "--seed", "12345", "--verbose"], cwd=tmp_path,
                             check=True, capture_output=True, text=True, env=env).stdout
        trace = [int(line.split(":")[1]) for line in out.splitlines() if line.startswith("Size of")]
        with open(tmp_path / "clustering_result.txt", "rb") as f:
            runs.append((trace, hashlib.md5(f.read()).hexdigest()))
    assert runs[0] == runs[1]
    trace = runs[0][0]
    assert len(trace) > 10 + 20000 // 3000  # init batches + re-cluster passes + the main loop
    assert trace[-10] <= 3000  # the main loop starts below the batch threshold
