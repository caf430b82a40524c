"""Mode B: the k-mer table built from KMC databases.

CPU: the oracle (oracle/klsh_oracle_b.py) reproduces the reference CLI's own outputs byte for byte
(tests/golden/mode_b.json: kmer_count.log verbatim and the md5s of kmer_set.hex / kmer_count.bin,
rows in the reference's libcuckoo table order), and the product's host replay of that table
(klsh_cuckoo_order, no GPU) gives the oracle's order, up to a table loaded to 95.6 % ("bl_fill").
GPU: klsh_build_khtable writes the reference's three files byte for byte.
"""
import hashlib
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
ALL_CASES = CASES + ["bl_fill"]


def fixtures():
    with open(os.path.join(GOLDEN, "mode_b.json")) as f:
        return json.load(f)


def write(case, path):
    return (ki.write_big_case if case in ki.BIG_CASES else ki.write_case)(str(path), case)


def rows_md5(reps, counts):
    """md5s of kmer_set.hex and kmer_count.bin as the reference writes them from these rows."""
    hx = hashlib.md5(np.ascontiguousarray(reps, "<u8").tobytes()).hexdigest()
    bn = hashlib.md5(np.ascontiguousarray(counts, "<u2").tobytes()).hexdigest()
    return hx, bn


@pytest.mark.parametrize("case", ALL_CASES)
def test_oracle_mode_b_matches_reference(case, tmp_path):
    """KMC1 and KMC2 (3 signature bins) layouts, min_count filtering (the all-A k-mer the
    reference then adds), 65535 saturation, databases listing both strands, and a 501K-k-mer
    table at 95.6 % load: the oracle's rows are the reference's files byte for byte."""
    info = write(case, tmp_path)
    fx = fixtures()[case]
    reps, counts, log = ob.build_khtable([str(tmp_path / n) for n in info["names"]], info["k"])
    reps = np.array(reps, np.uint64)
    assert log == fx["log"]
    assert len(reps) == fx["kmap"]
    assert rows_md5(reps, counts) == (fx["hex_md5"], fx["bin_md5"])
    assert row_digest(reps, counts) == fx["rows_md5"]
    assert int((counts == 65535).sum()) == fx["saturated"]
    assert (0 in reps) == fx["has_zero_kmer"]


@pytest.mark.parametrize("case", ALL_CASES)
def test_host_cuckoo_order_matches_oracle(case, tmp_path):
    """The product's host replay of the reference's libcuckoo inserts (klsh_cuckoo_order, no GPU)
    orders the first-appearance rows exactly as the oracle does."""
    from kmerlsh_amd import _native

    info = write(case, tmp_path)
    first, _, _ = ob.build_khtable([str(tmp_path / n) for n in info["names"]], info["k"],
                                   order="first")
    idx, hp = ob.cuckoo_order(first, info["k"])
    mine, mhp = _native.cuckoo_order(np.array(first, np.uint64), info["k"])
    assert mhp == hp == 16
    assert np.array_equal(mine, np.array(idx, np.uint32))


def test_cuckoo_order_grows_like_a_sequential_table():
    """Past 2^16 x 8 slots the table doubles; the reference re-inserts from several threads (its
    order is then not reproducible run to run), the product as those threads would one after
    another — the same as the oracle's sequential restatement."""
    from kmerlsh_amd import _native

    rng = np.random.default_rng(5)
    reps = np.unique(rng.integers(0, 1 << 62, 530_000, dtype=np.uint64))
    rng.shuffle(reps)
    idx, hp = ob.cuckoo_order(list(reps), 31)
    mine, mhp = _native.cuckoo_order(reps, 31)
    assert hp == mhp == 17
    assert np.array_equal(mine, np.array(idx, np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ALL_CASES)
def test_build_khtable_matches_reference(engine, case, tmp_path):
    info = write(case, tmp_path)
    fx = fixtures()[case]
    st = engine.build_khtable([str(tmp_path / n) for n in info["names"]], info["k"], str(tmp_path))
    assert st["kmap_size"] == fx["kmap"]
    with open(tmp_path / "kmer_count.log") as f:
        assert f.read() == fx["log"]
    for name, key in (("kmer_set.hex", "hex_md5"), ("kmer_count.bin", "bin_md5")):
        with open(tmp_path / name, "rb") as f:
            assert hashlib.md5(f.read()).hexdigest() == fx[key], name


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
