"""Mode E: the differential test of the clusters and the read extraction.

CPU (`-m "not gpu"`): the product's host pieces against fixtures the reference made —
ALGLIB's t-test bits (tests/golden/ttest.npz), the FASTQ record rules, the per-cluster groups —
and the oracle (oracle/klsh_oracle_e.py) against the reference CLI's own outputs
(tests/golden/mode_e.json).  GPU (`-m gpu`): the k-mer vote kernel and the whole mode-E command
line through the C ABI, bit-exact against the oracle and the reference's output md5s.
"""
import gzip
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, golden

import klsh_oracle_e as oe  # noqa: E402  (oracle/ is on sys.path via conftest)

import sys

sys.path.insert(0, GOLDEN)
import mode_e_inputs as mi  # noqa: E402

CASES = sorted(mi.CASES)


def fixtures():
    with open(os.path.join(GOLDEN, "mode_e.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def case_dirs(tmp_path_factory):
    out = {}
    for c in CASES:
        p = tmp_path_factory.mktemp(c)
        mi.write_case(str(p), c)
        out[c] = str(p)
    return out


# ------------------------------------------------------------------------------------ CPU ----
def test_ttest_bits_match_alglib():
    """klsh_ttest2 (host restatement of alglib::studentttest2 and the Cephes functions under it)
    against ALGLIB itself: 640 cases incl. constant groups, tiny/huge spreads, t < -2 (incomplete
    beta), n or m = 0 / 1 (statistics.cpp:12502-12620)."""
    from kmerlsh_amd import _native

    z = golden("ttest.npz")
    groups = len([f for f in z.files if f.startswith("v")])
    for g in range(groups):
        v, (n, m), t = z["v%d" % g], z["nm%d" % g], z["t%d" % g]
        for c in range(v.shape[0]):
            got = np.array(_native.ttest2(v[c, :n].astype(np.float64), v[c, n:].astype(np.float64)))
            assert np.array_equal(got.view(np.uint64), t[c].view(np.uint64)), (g, c, got, t[c])


@pytest.mark.parametrize("case", CASES)
def test_oracle_mode_e_matches_reference(case, case_dirs):
    """The oracle's whole mode E reproduces the reference CLI's output files byte for byte."""
    c = mi.CASES[case]
    fx = fixtures()[case]
    outs, counts = oe.mode_e(case_dirs[case], c["k"], c["size_thresh"], c["pval"], c["vote"])
    assert list(counts) == fx["differential"]
    assert sorted(outs) == sorted(fx["files"])
    for name, blob in outs.items():
        assert hashlib.md5(blob).hexdigest() == fx["files"][name]["md5"], name


@pytest.mark.parametrize("case", CASES)
def test_fastq_reader_matches_oracle(case, case_dirs):
    """The product's FASTQ reader (host) gives the reference's records: CRLF names keep '\\r',
    multi-line records, gzip, the empty-sequence record, lowercase / N bases."""
    from kmerlsh_amd import _native

    d = case_dirs[case]
    for fn in sorted(os.listdir(d)):
        if ".fq" in fn and not fn.startswith(("A_", "B_")):
            p = os.path.join(d, fn)
            assert _native.fastq_records(p, batch=97) == oe.read_fastq(p), fn


def test_fastq_reader_edge_records(tmp_path):
    """kseq corner cases: blank lines and junk before '@', '@' inside the quality, a missing final
    newline, a truncated last record (ends the file), a 0xFF byte (reads as end of input)."""
    from kmerlsh_amd import _native

    texts = {
        "junk.fq": b"\n\njunk line\n@r1 a b\nACGT\n+\n@@@@\n\n\n@r2\nAC\nGT\n+x\nII\nII\n",
        "nofinalnl.fq": b"@r1\nACGTN\n+\n!!!!!\n@r2\nACG\n+\n###",
        "trunc.fq": b"@r1\nACGT\n+\nIIII\n@r2\nACGTACGT\n+\nIII\n",
        "ff.fq": b"@r1\nACGT\n+\nIIII\n\xff@r2\nACGT\n+\nIIII\n",
        "plus_in_seq.fq": b"@r1\nAC+GT\n+\nII\n@r2\nA\n+\nI\n",
    }
    for fn, blob in texts.items():
        p = tmp_path / fn
        p.write_bytes(blob)
        assert _native.fastq_records(str(p)) == oe.read_fastq(str(p)), fn
    gz = tmp_path / "junk.fq.gz"
    with gzip.open(gz, "wb") as f:
        f.write(texts["junk.fq"])
    assert _native.fastq_records(str(gz)) == oe.read_fastq(str(tmp_path / "junk.fq"))


@pytest.mark.parametrize("case", CASES)
def test_wrs_groups_match_oracle(case, case_dirs):
    """klsh_wrs (AB::WRS for every cluster) against the oracle's decisions, and the numbers of
    differential ids the reference printed."""
    from kmerlsh_amd import _native

    c = mi.CASES[case]
    d = c["n1"] + c["n2"]
    vals, id_lists = oe.read_cluster_all(os.path.join(case_dirs[case], "clustering_result.txt"), d)
    counts = np.array([len(x) for x in id_lists], np.uint64)
    g = _native.wrs(vals, counts, c["n1"], c["n2"], c["pval"], c["size_thresh"])
    assert np.array_equal(g, oe.wrs_groups(vals, id_lists, c["n1"], c["n2"], c["pval"],
                                           c["size_thresh"]))
    a = set().union(*[set(x) for x, gg in zip(id_lists, g) if gg == 1])
    b = set().union(*[set(x) for x, gg in zip(id_lists, g) if gg == 2])
    assert [len(a), len(b)] == fixtures()[case]["differential"]
    assert (g == 1).any() and (g == 2).any() and (g == 0).any()


def test_canonical_kmers_oracle_edges():
    """The oracle's k-mer images against direct restatements of set_kmer / twin / operator<."""
    rng = np.random.default_rng(5)
    for k in (1, 2, 3, 4, 5, 8, 15, 16, 17, 21, 31, 32):
        s = rng.choice(list(b"ACGTNacgt"), size=k + 40).astype(np.uint8).tobytes()
        reps = oe.canonical_kmers(s, k)
        for p in (0, 7, 40):
            v = mi.fwd_value(s[p:p + k].decode(), k)
            assert int(reps[p]) == mi.rep(v, k)


# ------------------------------------------------------------------------------------ GPU ----
@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_cli_mode_e_matches_reference(case, tmp_path):
    """kmerLSH -M E --only (GPU k-mer vote) writes the reference's files byte for byte."""
    from kmerlsh_amd import _native

    mi.write_case(str(tmp_path), case)
    fx = fixtures()[case]
    args = [a for a in mi.cli_args(case) if a not in ("-T", "1")]
    out = subprocess.run([_native.CLI_PATH] + args, cwd=tmp_path, check=True, capture_output=True,
                         text=True, timeout=300).stdout
    for name, f in fx["files"].items():
        with open(tmp_path / name, "rb") as fh:
            assert hashlib.md5(fh.read()).hexdigest() == f["md5"], name
    got = [int(line.split(":")[1]) for line in out.splitlines() if "# of differential" in line]
    assert got == fx["differential"]
    assert out.count("abnormal read entry skipped") == fx["abnormal"]


def random_reads(rng, n, kset_src, k):
    """Reads drawn partly from the set's k-mers' source sequences, with N / lowercase / junk
    characters and every length class around k + 10 (plus window-crossing long reads)."""
    reads = []
    for r in range(n):
        u = r % 10
        ln = (k + 9 if u == 0 else k + 10 if u == 1 else 5000 if u == 2 and r % 50 == 2
              else int(rng.integers(k + 10, k + 300)))
        if u in (3, 4, 5, 6) and len(kset_src) > ln:
            a = int(rng.integers(0, len(kset_src) - ln))
            s = bytearray(kset_src[a:a + ln])
        else:
            s = bytearray(rng.choice(list(b"ACGT"), size=ln).astype(np.uint8).tobytes())
        for q in rng.integers(0, ln, size=ln // 40):
            s[q] = int(rng.choice(list(b"NnacgtXY")))
        reads.append(bytes(s))
    return reads


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2, 5, 15, 21, 31, 32])
def test_check_reads_vs_oracle(engine, k):
    """Per-read k-mer hits and vote flags of the GPU kernel equal the oracle's, for k from 1 to
    32 (the whole 64-bit word), reads of k+9 / k+10 bases, reads longer than the 2048-position LDS
    window, non-ACGT characters."""
    from kmerlsh_amd import _native

    rng = np.random.default_rng(100 + k)
    src = rng.choice(list(b"ACGT"), size=20000).astype(np.uint8).tobytes()
    kset = np.unique(oe.canonical_kmers(src[:12000], k))
    kset = np.concatenate([kset, rng.integers(0, 2**63, size=500, dtype=np.uint64)])
    reads = random_reads(rng, 600, src, k)
    ks = _native.KmerSet(engine, kset)
    for vote in (0.5, 0.0, 0.99):
        hits, flags = ks.check_reads(reads, k, vote)
        oh, of = oe.check_reads(reads, kset, k, vote)
        assert np.array_equal(hits, oh), vote
        assert np.array_equal(flags, of), vote
    ks.close()


@pytest.mark.gpu
def test_check_reads_empty_set_and_no_reads(engine):
    from kmerlsh_amd import _native

    ks = _native.KmerSet(engine, np.zeros(0, np.uint64))
    hits, flags = ks.check_reads([b"ACGT" * 20, b""], 21, 0.0)
    assert hits.tolist() == [0, 0] and flags.tolist() == [0, 0]
    ks.close()
    ks = _native.KmerSet(engine, np.array([0xFFFFFFFFFFFFFFFF, 0], np.uint64))
    hits, flags = ks.check_reads([b"A" * 50, b"T" * 50], 32, 0.5)  # both canonical reps are 0
    assert hits.tolist() == [19, 19] and flags.tolist() == [1, 1]
    ks.close()


@pytest.mark.gpu
def test_extract_fastq_batches_match_single_call(engine, tmp_path):
    """klsh_extract_fastq over 300K reads (two parse batches of 2^18 in flight, gzip input)
    writes exactly the records whose one-call check_reads flag is set, in order."""
    from kmerlsh_amd import _native

    k, vote = 21, 0.4
    rng = np.random.default_rng(77)
    src = rng.choice(list(b"ACGT"), size=50000).astype(np.uint8).tobytes()
    kset = np.unique(oe.canonical_kmers(src[:30000], k))
    n = 300000
    starts = rng.integers(0, len(src) - 200, size=n)
    lens = rng.integers(20, 180, size=n)
    seqs = [src[a:a + ln] for a, ln in zip(starts.tolist(), lens.tolist())]
    lines = []
    for i, s in enumerate(seqs):
        lines.append(b"@q%d x\n%s\n+\n%s\n" % (i, s, b"I" * len(s)))
    path = tmp_path / "big.fq.gz"
    with gzip.open(path, "wb", compresslevel=1) as f:
        f.write(b"".join(lines))
    ks = _native.KmerSet(engine, kset)
    st = ks.extract_fastq(str(path), str(tmp_path / "out.fq"), k, vote)
    _, flags = ks.check_reads(seqs, k, vote)
    ks.close()
    expect = b"".join(lines[i] for i in np.nonzero(flags)[0])
    assert (tmp_path / "out.fq").read_bytes() == expect
    assert st["reads"] == n and st["reads_extracted"] == int(flags.sum())
    assert 0 < st["reads_extracted"] < n
