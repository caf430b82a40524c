"""Mode B: the k-mer table built from KMC databases.

CPU: the oracle (oracle/klsh_oracle_b.py) reproduces the reference CLI's own outputs
(tests/golden/mode_b.json: kmer_count.log verbatim and a digest of the rows keyed by k-mer — the
reference's row order is its libcuckoo table's, so rows are compared order-free).
GPU: klsh_build_khtable / `kmerLSH -M B --only` write the same log, the same rows (digest) and
rows in the oracle's first-appearance order, byte for byte.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN

import klsh_oracle_b as ob  # noqa: E402

sys.path.insert(0, GOLDEN)
import kmc_inputs as ki  # noqa: E402
from make_golden_b import row_digest  # noqa: E402

CASES = sorted(ki.CASES)


def fixtures():
    with open(os.path.join(GOLDEN, "mode_b.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", CASES)
def test_oracle_mode_b_matches_reference(case, tmp_path):
    """KMC1 and KMC2 (3 signature bins) layouts, min_count filtering (the all-A k-mer the
    reference then adds), 65535 saturation, databases listing both strands."""
    info = ki.write_case(str(tmp_path), case)
    fx = fixtures()[case]
    reps, counts, log = ob.build_khtable([str(tmp_path / n) for n in info["names"]], info["k"])
    assert log == fx["log"]
    assert len(reps) == fx["kmap"]
    assert row_digest(np.array(reps, np.uint64), counts) == fx["rows_md5"]
    assert int((counts == 65535).sum()) == fx["saturated"]
    assert (0 in reps) == fx["has_zero_kmer"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_build_khtable_matches_reference(engine, case, tmp_path):
    info = ki.write_case(str(tmp_path), case)
    fx = fixtures()[case]
    st = engine.build_khtable([str(tmp_path / n) for n in info["names"]], info["k"], str(tmp_path))
    reps, counts, log = ob.read_outputs(str(tmp_path), info["d"])
    assert log == fx["log"]
    assert st["kmap_size"] == fx["kmap"]
    assert row_digest(reps, counts) == fx["rows_md5"]
    o_reps, o_counts, _ = ob.build_khtable([str(tmp_path / n) for n in info["names"]], info["k"])
    assert np.array_equal(reps, np.array(o_reps, np.uint64))  # first-appearance order
    assert np.array_equal(counts, o_counts)


@pytest.mark.gpu
def test_cli_mode_b_then_cluster(tmp_path):
    """kmerLSH -M B --only, then -M C --only on its output (the B -> C hand-off)."""
    from kmerlsh_amd import _native

    ki.write_case(str(tmp_path), "b21")
    fx = fixtures()["b21"]
    args = [a for a in ki.cli_args("b21") if a not in ("-T", "1")]
    subprocess.run([_native.CLI_PATH] + args, cwd=tmp_path, check=True, capture_output=True,
                   timeout=300)
    with open(tmp_path / "kmer_count.log") as f:
        assert f.read() == fx["log"]
    subprocess.run([_native.CLI_PATH, "-a", "a.txt", "-b", "b.txt", "-I", "5", "-M", "C", "--only"],
                   cwd=tmp_path, check=True, capture_output=True, timeout=300)
    assert os.path.getsize(tmp_path / "clustering_result.txt") > 0
