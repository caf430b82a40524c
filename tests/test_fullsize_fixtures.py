"""The full-size fixtures themselves (CPU): every bench workload is pinned over its whole loop, and
the headline (C2) and C1 are pinned to the seeded reference CLI's own run, not only the oracle's.

tests/golden/make_fullsize.py made them (the oracle, and with --reference the reference CLI at
-T 1 on the same count files); tests/test_gpu_fullsize.py checks the GPU engine against them.
"""
import glob
import json
import os

import pytest

from conftest import GOLDEN

FIXTURES = sorted(os.path.basename(p)[len("fullsize_"):-len(".json")]
                  for p in glob.glob(os.path.join(GOLDEN, "fullsize_*.json")))


def fixture(name):
    with open(os.path.join(GOLDEN, f"fullsize_{name}.json")) as f:
        return json.load(f)


def test_every_config_has_a_fixture():
    assert set(FIXTURES) >= {"c1", "c2", "c4", "c5"}


@pytest.mark.parametrize("name", FIXTURES)
def test_whole_loop_pinned(name):
    fx = fixture(name)
    assert fx["run_iterations"] == fx["iterations"]
    assert len(fx["trace"]) == fx["iterations"]
    assert sum(fx["trace"]) == fx["sum_trace"]
    assert all(a >= b for a, b in zip(fx["trace"], fx["trace"][1:]))
    assert fx["trace"][0] == fx["n_init"] and fx["n_final"] <= fx["trace"][-1]
    assert set(fx["written_md5"]) == {"clustering_result.txt", "clustering_result.txt.clust"}


@pytest.mark.parametrize("name", ["c1", "c2"])
def test_reference_cli_agrees(name):
    """The seeded reference CLI (oracle/_ref/kmerLSH_seeded, -T 1, mode C) on the same count files:
    the init-pass and main-loop N_t traces and both output files equal the oracle's."""
    fx = fixture(name)
    ref = fx["reference"]
    assert ref["agrees"]
    assert ref["trace"] == fx["trace"]
    assert ref["init_trace"] == fx["init_trace"]
    assert ref["md5"] == fx["written_md5"]
