"""Parity of the gfx950 engine (through the C ABI) with the reference and the oracle.

Bar: bit-exact.  Keys, survivor order, member-id lists, N_t traces and the fp32 centroid bits
must all equal the reference's outputs (golden fixtures made by the reference itself) and the
oracle's on the same seeded inputs; at full size, size-independent properties are checked.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, golden

pytestmark = pytest.mark.gpu

sys.path.insert(0, GOLDEN)


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a, np.float32).view(np.uint32),
                          np.ascontiguousarray(b, np.float32).view(np.uint32))


def assert_same_result(got, rows, off, ids):
    g_rows, g_off, g_ids = got
    assert np.array_equal(g_off, off)
    assert np.array_equal(g_ids, ids)
    assert same_bits(g_rows, rows)


# --------------------------------------------------------------------------- arithmetic ------
def test_fp_sqrt_div_correctly_rounded(engine):
    rng = np.random.default_rng(1)
    a = np.concatenate([rng.random(200000).astype(np.float32) * 1e4,
                        rng.random(20000).astype(np.float32) * np.float32(1e-38),  # subnormal
                        np.array([0, 1, 2, 3, 4, 1e30, 3.4e38], np.float32)])
    b = np.concatenate([rng.random(a.size - 7).astype(np.float32) * 100 + 1e-3,
                        np.array([1, 3, 7, 0.1, 9, 1e-30, 0.5], np.float32)])
    s, q = engine.fp_selftest(a, b)
    assert same_bits(s, np.sqrt(a))
    assert same_bits(q, a / b)


@pytest.mark.parametrize("name", ["keys_d8", "keys_d16", "keys_d64", "keys_d13", "keys_d512"])
def test_hash_keys_match_reference(engine, name):
    from kmerlsh_amd import _native

    z = golden(name + ".npz")
    w, _ = _native.hyperplanes(int(z["seed"]), 0, int(z["h"]), z["rows"].shape[1])
    assert np.array_equal(engine.hash_keys(z["rows"], w), z["keys"])


@pytest.mark.parametrize("n,bits,spread", [
    (1, 8, 1), (2, 1, 2), (2047, 8, 300), (2048, 13, 1 << 13), (2049, 16, 5),
    (100_000, 17, 1 << 17), (300_000, 23, 1000), (1_000_003, 22, 1 << 22), (5_000_000, 23, 1 << 23),
    (200_000, 31, 1 << 31), (70_000, 0, 1),
    (390_000, 18, 1 << 18), (1_500_000, 20, 1 << 20), (300_000, 19, 700), (150_000, 17, 1 << 17),
])
def test_bucket_sort_is_stable_counting_sort(engine, n, bits, spread):
    """merge_hashtable (cluster.cc:15-30) scatters rows into lsh_table[key] in row order: the
    stable bucket order, i.e. numpy's stable argsort of the keys (single-pass look-back sort)."""
    rng = np.random.default_rng(n + bits)
    keys = rng.integers(0, spread, n, dtype=np.uint64).astype(np.uint32)
    if bits < 32:
        keys &= np.uint32((1 << bits) - 1) if bits else np.uint32(0)
    got_k, got_p = engine.bucket_sort(keys, bits)
    want = np.argsort(keys, kind="stable")
    assert np.array_equal(got_p, want.astype(np.uint32))
    assert np.array_equal(got_k, keys[want])


def test_bucket_sort_repeated_calls(engine):
    """several sorts of different sizes in a row on one context"""
    rng = np.random.default_rng(5)
    for n in (300_000, 4_096, 1, 2_500_000, 65_537):
        keys = rng.integers(0, 1 << 20, n, dtype=np.uint32)
        k, p = engine.bucket_sort(keys, 20)
        assert np.array_equal(p, np.argsort(keys, kind="stable").astype(np.uint32))


def test_hash_keys_random_vs_oracle(engine, oracle):
    from kmerlsh_amd import _native

    rng = np.random.default_rng(3)
    for d, h in [(32, 17), (64, 31), (8, 1), (5, 7), (100, 20)]:
        rows = rng.normal(0, 1, size=(3000, d)).astype(np.float32)
        w, _ = _native.hyperplanes(99 + d, 5, h, d)
        assert np.array_equal(engine.hash_keys(rows, w), oracle.keys(rows, w)), (d, h)


def adversarial_rows(rng, n, d, w):
    """Rows the certified projection screens cannot call, and rows that break the fp16 image:
    every third row projected onto hyperplane i % h (s is rounding noise around 0), rows whose
    sequential sum is exactly 0 for a hyperplane (x = w_l e_k - w_k e_l: the two products are
    exact negatives), zero / -0 / tiny / huge / NaN / inf rows, elements past fp16's range
    (>= 65520 -> inf in the image), fp16-subnormal rows and rows whose fp16 image is all zero
    while the f32 row is not, f32-subnormal rows."""
    h = w.shape[0]
    w64 = w.astype(np.float64)
    rows = rng.normal(0, 1, size=(n, d))
    for i in range(0, n, 3):
        j = i % h
        rows[i] -= (rows[i] @ w64[j]) / (w64[j] @ w64[j]) * w64[j]
    rows = rows.astype(np.float32)
    f = np.float32
    rows[1] = 0.0
    rows[4] *= f(1e-30)
    rows[7] *= f(1e30)
    rows[10, 3] = np.nan
    rows[13] = -0.0
    for m, i in enumerate(range(2, min(n, 2 + 3 * h * 4), 3)):  # s == 0 exactly for hyperplane j
        j, k = m % h, (m * 7) % d
        l = (k + 1 + m % (d - 1)) % d if d > 1 else k
        if l == k:
            continue
        rows[i] = 0.0
        rows[i, k], rows[i, l] = w[j, l], -w[j, k]
        if m % 2:
            rows[i] *= f(-1)
    special = {
        16: lambda r: r.__setitem__(0, f(70000.0)),      # fp16 overflow: inf in the image
        19: lambda r: r.__setitem__(d - 1, f(65519.0)),  # rounds to 65504, finite
        22: lambda r: r.__imul__(f(1e-6)),               # fp16 subnormal image
        25: lambda r: r.__imul__(f(1e-9)),               # fp16 image all zero, f32 nonzero
        28: lambda r: r.__setitem__(slice(0, d // 2), r[: d // 2] * f(1e-9)),
        31: lambda r: r.__setitem__(slice(None), np.where(np.arange(d) % 2, f(-0.0), f(0.0))),
        34: lambda r: r.__setitem__(0, f(np.inf)),
        37: lambda r: r.__imul__(f(1e-40)),              # f32 subnormal
        40: lambda r: r.__setitem__(slice(None), f(65504.0)),
        43: lambda r: r.__setitem__(d // 2, f(-1e5)),
    }
    for i, fn in special.items():
        if i < n:
            fn(rows[i])
    return rows


@pytest.mark.parametrize("d,h", [(64, 23), (32, 18), (16, 9), (64, 31), (32, 1), (8, 7), (512, 20),
                                 (100, 31), (72, 5), (136, 31)])
def test_hash_keys_close_calls_vs_oracle(engine, oracle, d, h):
    """The loop's projection kernels (klsh_hash_keys uses the same dispatch: the fp16 row image
    at d = 16/32/64, the f32 fp16x3 screen above 64) on adversarial rows, bit-equal to the
    reference's sequential chains (hash/lshash.cc:44-59: s == +0/-0 -> 1, tiny negative -> 0,
    NaN -> 0).  The screen runs and leaves close calls to the exact chains, which the test
    asserts."""
    from kmerlsh_amd import _native

    rng = np.random.default_rng(11 + d + h)
    w, _ = _native.hyperplanes(7 + d, 0, h, d)
    rows = adversarial_rows(rng, 4000, d, w)
    got = engine.hash_keys(rows, w)
    kern = engine.get_option("last_hash_kernel")
    assert np.array_equal(got, oracle.keys(rows, w)), (d, h)
    # fp16 screen / packed / f32 fp16x3 wide screen
    want = {16: 1, 32: 1, 64: 1, 8: 0}.get(d, 2)
    assert kern == want, kern
    if kern:
        assert engine.get_option("last_hash_close_pairs") > 0


@pytest.mark.parametrize("segcap", [1, 3])
def test_hash_keys_fp16_fixup_segment_full(engine, oracle, segcap):
    """k_project_h16's fix-up segment filled up (a test-only cap of 1 or 3 entries per workgroup):
    the close calls past it are settled in place by the exact chain, same bits."""
    from kmerlsh_amd import _native

    engine.set_option("h16_segcap", segcap)
    try:
        for d, h in [(64, 23), (32, 17), (16, 12)]:
            w, _ = _native.hyperplanes(3 + d, 0, h, d)
            rows = adversarial_rows(np.random.default_rng(d), 9000, d, w)
            assert np.array_equal(engine.hash_keys(rows, w), oracle.keys(rows, w)), (d, h)
            assert engine.get_option("last_hash_kernel") == 1
    finally:
        engine.set_option("h16_segcap", 0)


def test_hash_keys_packed_variant(engine, oracle):
    """Option "projection" = 1: the exact packed VALU chains at every width, the same keys."""
    from kmerlsh_amd import _native

    engine.set_option("projection", 1)
    try:
        for d, h in [(64, 23), (32, 31), (16, 9), (100, 20)]:
            w, _ = _native.hyperplanes(7 + d, 0, h, d)
            rows = adversarial_rows(np.random.default_rng(d), 5000, d, w)
            assert np.array_equal(engine.hash_keys(rows, w), oracle.keys(rows, w)), (d, h)
            assert engine.get_option("last_hash_kernel") == 0
    finally:
        engine.set_option("projection", 0)


@pytest.mark.parametrize("n,d,groups,noise", [(120000, 64, 1500, 0.05), (600000, 32, 20000, 0.05),
                                               (200000, 16, 50, 0.01), (3000, 64, 100, 0.05),
                                               (1048000, 8, 30000, 0.1), (1900, 32, 1700, 0.05)])
def test_tail_local_sort_vs_oracle(engine, oracle, n, d, groups, noise):
    """The queued small iterations' bucket sort as a top-9-bit partition (kTailTopBits) + per-bucket
    LDS sorts of the remaining 1..10 bits that list the runs (option tail_local, default) and as the
    LSD passes + run kernels: both equal the oracle (merge_hashtable's stable order,
    cluster.cc:15-30), buckets over 4096 keys (several LDS rounds) included.  tail_local_ok takes
    keys of 10..19 bits: 1900 rows of 1700 groups stay in [1024, 2048) rows, so every queued
    iteration has 10-bit keys (one low bit per top bucket), and the 1048000-row case starts at
    19 bits."""
    rng = np.random.default_rng(n + d)
    rows = clustered(rng, n, d, groups, noise)
    want = oracle.cluster(rows, 0.8, 8, 1000000, 41, 9)
    try:
        for local in (1, 0):
            engine.set_option("tail_local", local)
            engine.load_rows(rows)
            trace, counter, _ = engine.cluster(0.8, 8, 1000000, 41, 9)
            assert np.array_equal(trace, want[3]) and counter == want[4], local
            assert_same_result(engine.result(), *want[:3])
    finally:
        engine.set_option("tail_local", 1)


@pytest.mark.parametrize("n,d,groups,noise,with_oracle", [(1500000, 16, 30000, 0.05, True),
                                                           (2600000, 32, 60000, 0.05, False)])
def test_mid_local_sort(engine, oracle, n, d, groups, noise, with_oracle):
    """Iterations of 2^20 .. 2^22 positions (20- and 21-bit keys: the host-driven path with the
    one-launch merge) then the queued tail, with option tail_local on and off — the same trace,
    counter and result bits, and the oracle's for the smaller case.  (A top-10-bit partition +
    LDS bucket sorts for these keys measured slower than the LSD passes, C2 186.5 -> 188.5 ms,
    and was not kept.)"""
    rng = np.random.default_rng(n + d)
    rows = clustered(rng, n, d, groups, noise)
    got = []
    try:
        for local in (1, 0):
            engine.set_option("tail_local", local)
            engine.load_rows(rows)
            trace, counter, _ = engine.cluster(0.8, 3, 1000000, 41, 9)
            got.append((trace, counter, engine.result()))
    finally:
        engine.set_option("tail_local", 1)
    assert np.array_equal(got[0][0], got[1][0]) and got[0][1] == got[1][1]
    assert_same_result(got[0][2], *got[1][2])
    if with_oracle:
        want = oracle.cluster(rows, 0.8, 3, 1000000, 41, 9)
        assert np.array_equal(got[0][0], want[3]) and got[0][1] == want[4]
        assert_same_result(got[0][2], *want[:3])


@pytest.mark.parametrize("d", [64, 32])
def test_cluster_variants_agree(engine, oracle, d):
    """Options that change the launch sequence, not the result: the queued tail batches
    ("tail_batch") and the fp16-image projection ("projection") in all four combinations give the
    same N_t trace, RNG counter, statistics that count work, and result bits as the oracle."""
    rng = np.random.default_rng(d + 1)
    rows = clustered(rng, 120000, d, 1500, 0.05)
    want = oracle.cluster(rows, 0.8, 14, 1000000, 91, 2)
    seen = []
    try:
        for tail_batch in (1, 0):
            for proj in (0, 1):
                engine.set_option("tail_batch", tail_batch)
                engine.set_option("projection", proj)
                engine.load_rows(rows)
                assert engine.get_option("fp16_image") == (proj == 0)
                trace, counter, st = engine.cluster(0.8, 14, 1000000, 91, 2)
                assert np.array_equal(trace, want[3]) and counter == want[4], (tail_batch, proj)
                assert_same_result(engine.result(), *want[:3])
                assert st["project_launches"] == st["iterations"] == 14
                seen.append((st["iterations"], st["sum_merges"], st["hyperplanes"],
                             st["sum_rows"], st["sum_proj_bits"]))
    finally:
        engine.set_option("tail_batch", 1)
        engine.set_option("projection", 0)
    assert len(set(seen)) == 1, seen


def runs_reference(keys, bucket_thr):
    """Runs of equal keys (the buckets merge_hashtable fills, cluster.cc:15-30) of 2+ rows with the
    merge step's list: size class by length, > bucket_thr = nestedCluster (cluster.cc:286)."""
    n = keys.size
    heads = np.flatnonzero(np.concatenate([[True], keys[1:] != keys[:-1]])) if n else np.zeros(0, int)
    lens = np.diff(np.concatenate([heads, [n]]))
    keep = lens >= 2
    heads, lens = heads[keep], lens[keep]
    lists = np.empty(lens.size, np.int32)
    for i, b in enumerate(lens):
        if bucket_thr >= 0 and b > bucket_thr:
            lists[i] = 11
        elif b > 896:
            lists[i] = 10
        elif b > 64:
            lists[i] = 6 + int(np.searchsorted([128, 192, 384, 896], b))
        else:
            lists[i] = int(np.searchsorted([2, 4, 8, 16, 32, 64], b))
    return heads.astype(np.uint32), lens.astype(np.uint32), lists


@pytest.mark.parametrize("case", ["random", "giant", "giant_over", "tile_edges", "all_equal",
                                  "singletons", "long_mixed", "fused_giant"])
def test_bucket_runs_vs_reference(engine, case):
    """Run finding at any run length (a 4.2M-key run spans ~1000 tiles: linear, no per-tile
    forward walk), oversize runs (nestedCluster's list), runs ending exactly on tile edges; both
    the fused (<= 256 tiles) and the scanned path."""
    rng = np.random.default_rng(len(case))
    thr = -1
    if case == "random":
        keys = np.sort(rng.integers(0, 200_000, 1_500_000)).astype(np.uint32)
    elif case in ("giant", "giant_over"):
        keys = np.sort(np.concatenate([rng.integers(0, 1 << 20, 800_000),
                                       np.full(4_200_000, 777_777)])).astype(np.uint32)
        thr = 1_000_000 if case == "giant_over" else -1
    elif case == "tile_edges":
        lens = rng.choice([1, 2, 63, 64, 65, 896, 897, 4095, 4096, 4097, 8192], 3000)
        keys = np.repeat(np.arange(lens.size, dtype=np.uint32), lens)
        thr = 4096
    elif case == "all_equal":
        keys = np.zeros(3_000_000, np.uint32)
    elif case == "singletons":
        keys = np.arange(2_000_000, dtype=np.uint32)
    elif case == "long_mixed":
        lens = rng.integers(1, 20000, 400)
        keys = np.repeat(np.arange(lens.size, dtype=np.uint32) * 3, lens)
        thr = 9000
    else:  # fused: <= 256 tiles with a run across all of them
        keys = np.concatenate([np.zeros(5, np.uint32), np.full(900_000, 9, np.uint32),
                               np.arange(10, 100_010, dtype=np.uint32)])
    got = engine.bucket_runs(keys, thr)
    want = runs_reference(keys, thr)
    for g, w_ in zip(got, want):
        assert np.array_equal(g, w_), case


# ------------------------------------------------------------------------------ p_cluster ---
@pytest.mark.parametrize("name", ["pcluster_small", "pcluster_large", "pcluster_generic",
                                  "pcluster_d8"])
def test_pcluster_matches_reference(engine, name):
    z = golden(name + ".npz")
    engine.load_rows(z["rows"])
    engine.pcluster(float(z["thr"]))
    assert_same_result(engine.result(), z["out_rows"], z["out_off"], z["out_ids"])


@pytest.mark.parametrize("b,d,groups,noise,thr", [
    (65, 64, 6, 0.05, 0.9), (200, 32, 12, 0.08, 0.85), (384, 64, 30, 0.05, 0.95),
    (385, 64, 30, 0.05, 0.95), (700, 16, 50, 0.1, 0.8), (64, 8, 3, 0.2, 0.9), (3, 64, 1, 0.01, 0.9),
    (128, 64, 10, 0.05, 0.9), (129, 64, 10, 0.05, 0.9), (896, 64, 200, 0.05, 0.95),
    (897, 32, 200, 0.05, 0.95), (600, 8, 40, 0.1, 0.85), (250, 16, 1, 0.0, 0.9),
    # wide rows (chunked kernels): every size class, widths with and without partial chunks
    (2, 512, 1, 0.05, 0.9), (7, 512, 2, 0.05, 0.9), (33, 512, 4, 0.05, 0.9),
    (64, 100, 5, 0.05, 0.9), (100, 512, 8, 0.05, 0.9), (300, 130, 20, 0.05, 0.9),
    (500, 512, 30, 0.05, 0.95), (1000, 70, 60, 0.05, 0.9), (40, 13, 3, 0.1, 0.85),
    (60, 2048, 4, 0.05, 0.9),
    # > 896 rows (k_merge_huge, batched candidates): merge-sparse and merge-dense walks
    (3000, 32, 100, 0.05, 0.9), (2500, 64, 300, 0.08, 0.85), (1500, 16, 20, 0.03, 0.95),
    (4000, 8, 400, 0.1, 0.8), (1200, 32, 1200, 0.3, 0.99), (2000, 64, 2, 0.01, 0.9),
    # the 129..192 / 193..384 class boundary (two workgroups per CU below it)
    (192, 64, 15, 0.05, 0.9), (193, 64, 15, 0.05, 0.9), (160, 32, 1, 0.0, 0.9), (190, 16, 12, 0.1, 0.85),
    (180, 130, 12, 0.05, 0.9),
])
def test_pcluster_run_lengths_vs_oracle(engine, oracle, b, d, groups, noise, thr):
    """Every merge path by bucket length: G-lane groups (<= 64), LDS matrix (65..384), wave (> 384)."""
    rng = np.random.default_rng(b * 7 + d)
    rows = clustered(rng, b, d, groups, noise)
    engine.load_rows(rows)
    engine.pcluster(thr)
    assert_same_result(engine.result(), *oracle.pcluster(rows, thr))


@pytest.mark.parametrize("b,d,groups,noise,thr,long_runs", [
    (3000, 32, 100, 0.05, 0.9, 1), (3000, 32, 100, 0.05, 0.9, 0), (2500, 64, 300, 0.08, 0.85, 4),
    (1500, 16, 20, 0.03, 0.95, 1), (1500, 16, 20, 0.03, 0.95, 0), (1200, 512, 40, 0.05, 0.9, 4),
    (9000, 8, 900, 0.1, 0.8, 4), (2000, 100, 2, 0.01, 0.9, 4)])
def test_pcluster_huge_runs_folded_vs_oracle(engine, oracle, b, d, groups, noise, thr, long_runs):
    """Runs over 896 rows walked by the 385..896-row kernel's 256-lane workgroups (option
    "huge_fold", what the loop does after iterations without such runs) instead of k_merge_huge
    — through the per-class launches (tail_merge_rows = 1: k_merge_tail has no fold), and at
    d = 16 / 32 with k_merge_long off for them (long_runs 1: only >896-row runs would be its;
    0: none), which is where the fold takes over there."""
    rng = np.random.default_rng(b * 3 + d)
    rows = clustered(rng, b, d, groups, noise)
    with options(engine, huge_fold=1, tail_merge_rows=1, long_runs=long_runs):
        engine.load_rows(rows)
        engine.pcluster(thr)
        got = engine.result()
    assert_same_result(got, *oracle.pcluster(rows, thr))


class options:
    """Engine options set for a block and restored to their previous values after it."""

    def __init__(self, engine, **kv):
        self.engine, self.kv, self.old = engine, kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = self.engine.get_option(k)
            self.engine.set_option(k, v)
        return self.engine

    def __exit__(self, *exc):
        for k, v in self.old.items():
            self.engine.set_option(k, v)
        return False


@pytest.mark.parametrize("d,screen", [(64, 1), (32, 1), (64, 0)])
def test_small_screen_vs_oracle(engine, oracle, d, screen):
    """Option small_screen (default 1): runs of 2..64 rows screened on the fp16 row image first
    (only the ones the certified margin cannot rule out are merged on the f32 rows) — the same N_t
    trace, counter and result bits as the oracle, with rows the image cannot screen in small runs:
    past fp16's range, all-zero image of a nonzero row, zero, NaN; screen = 0: every small run
    through the f32 merge."""
    rng = np.random.default_rng(d + 7)
    rows = clustered(rng, 150000, d, 3000, 0.05)
    rows[5] *= np.float32(1e5)      # fp16 overflow in the image
    rows[9, 1] = np.float32(7e4)
    rows[11] *= np.float32(1e-9)    # image all zero
    rows[13] = 0.0
    rows[17, 2] = np.nan
    want = oracle.cluster(rows, 0.8, 12, 1000000, 93, 4)
    # tail_merge_rows = 1: every iteration through the per-class launches
    with options(engine, small_screen=screen, tail_merge_rows=1):
        engine.load_rows(rows)
        trace, counter, st = engine.cluster(0.8, 12, 1000000, 93, 4)
        got = engine.result()
    assert st["kern"]["screen"]["launches"] == 12 * screen
    assert np.array_equal(trace, want[3]) and counter == want[4]
    assert_same_result(got, *want[:3])


@pytest.mark.parametrize("b,d,groups,noise,thr", [
    (897, 32, 60, 0.05, 0.9), (1000, 16, 1000, 0.3, 0.99), (1536, 32, 100, 0.05, 0.9),
    (1537, 32, 100, 0.05, 0.9), (2048, 16, 150, 0.05, 0.9), (3000, 32, 300, 0.08, 0.85),
    (4096, 32, 50, 0.03, 0.95), (4097, 32, 400, 0.05, 0.9), (2500, 32, 2, 0.01, 0.9),
    (1800, 16, 1800, 0.5, 0.999), (1300, 32, 20, 0.2, 0.8), (5656, 32, 400, 0.05, 0.9),
    (8192, 32, 300, 0.05, 0.9), (6000, 16, 4, 0.01, 0.9), (7000, 32, 7000, 0.5, 0.999),
    (8193, 32, 400, 0.05, 0.9)])
def test_long_runs_vs_oracle(engine, oracle, b, d, groups, noise, thr):
    """Runs over 896 rows through k_merge_long (d = 16, 32: the Gram bit matrix in memory, one
    walk step per merge; rows past 1536 / 2048 positions read from memory; over 4096 rows:
    huge_runs in the same launch, up to C4's longest, 5656): merge-dense and merge-sparse, every
    length boundary."""
    rng = np.random.default_rng(b * 11 + d)
    rows = clustered(rng, b, d, groups, noise)
    with options(engine, tail_merge_rows=1):  # the per-class launches, not k_merge_tail
        engine.load_rows(rows)
        engine.pcluster(thr)
        got = engine.result()
    assert_same_result(got, *oracle.pcluster(rows, thr))


@pytest.mark.parametrize("b,d,groups,noise,thr", [
    (385, 32, 30, 0.05, 0.95), (700, 16, 50, 0.1, 0.8), (896, 32, 200, 0.05, 0.95),
    (640, 32, 640, 0.3, 0.99), (500, 32, 3, 0.02, 0.9)])
def test_long_runs_385_896_vs_oracle(engine, oracle, b, d, groups, noise, thr):
    """Option long_runs = 4: the 385..896-row runs through k_merge_long too (after the longer
    ones, in the same launch)."""
    rng = np.random.default_rng(b * 13 + d)
    rows = clustered(rng, b, d, groups, noise)
    with options(engine, tail_merge_rows=1, long_runs=4):
        engine.load_rows(rows)
        engine.pcluster(thr)
        got = engine.result()
    assert_same_result(got, *oracle.pcluster(rows, thr))


@pytest.mark.parametrize("special", ["nan", "zero", "huge", "tiny"])
def test_long_runs_special_rows(engine, oracle, special):
    """A long run with a row the pre-screen cannot call (NaN, zero, 1e30, 1e-30 scale): the
    exact chains decide it, in the Gram tiles and in the walk."""
    rng = np.random.default_rng(5)
    rows = clustered(rng, 1200, 32, 80, 0.05)
    k = 600
    if special == "nan":
        rows[k, 3] = np.nan
    elif special == "zero":
        rows[k] = 0.0
    elif special == "huge":
        rows[k] *= np.float32(1e30)
    else:
        rows[k] *= np.float32(1e-30)
    with options(engine, tail_merge_rows=1):
        engine.load_rows(rows)
        engine.pcluster(0.9)
        got = engine.result()
    assert_same_result(got, *oracle.pcluster(rows, 0.9))


@pytest.mark.parametrize("b,groups,noise,thr", [
    (193, 15, 0.05, 0.9), (384, 30, 0.05, 0.95), (384, 384, 0.3, 0.99), (385, 30, 0.05, 0.95),
    (385, 3, 0.02, 0.9), (640, 640, 0.3, 0.99), (896, 200, 0.05, 0.95), (896, 2, 0.01, 0.9)])
@pytest.mark.parametrize("per_class", [1, 0])
def test_big_runs_d64_vs_oracle(engine, oracle, b, groups, noise, thr, per_class):
    """d = 64 (C2's width) runs at the 193..384 / 385..896 class edges, merge-dense (one group
    per row at a high threshold: few merges, many decisions near s*) and merge-sparse or dense
    (few groups), through the per-class launches (k_merge_big<64, 384 / 896>, tail_merge_rows = 1)
    and through k_merge_tail's big-run workgroups (the default at these sizes)."""
    rng = np.random.default_rng(b * 17 + groups)
    rows = clustered(rng, b, 64, groups, noise)
    with options(engine, tail_merge_rows=1 if per_class else 0):
        engine.load_rows(rows)
        engine.pcluster(thr)
        got = engine.result()
    assert_same_result(got, *oracle.pcluster(rows, thr))


@pytest.mark.parametrize("special", ["nan", "zero", "huge", "tiny"])
@pytest.mark.parametrize("b", [385, 896])
def test_big_runs_d64_special_rows(engine, oracle, special, b):
    """A 385- / 896-row run at d = 64 with a row the Gram pre-screen cannot call (NaN, zero,
    1e30, 1e-30 scale): the exact chains decide it, in the tiles and in the walk, through both
    launch paths."""
    rng = np.random.default_rng(b)
    rows = clustered(rng, b, 64, 40, 0.05)
    k = b // 2
    if special == "nan":
        rows[k, 3] = np.nan
    elif special == "zero":
        rows[k] = 0.0
    elif special == "huge":
        rows[k] *= np.float32(1e30)
    else:
        rows[k] *= np.float32(1e-30)
    want = oracle.pcluster(rows, 0.9)
    for per_class in (1, 0):
        with options(engine, tail_merge_rows=1 if per_class else 0):
            engine.load_rows(rows)
            engine.pcluster(0.9)
            got = engine.result()
        assert_same_result(got, *want)


@pytest.mark.parametrize("n,groups,noise", [(200000, 100, 0.03), (300000, 120, 0.3)])
def test_long_runs_many_at_once_vs_oracle(engine, oracle, n, groups, noise):
    """Hundreds of runs over 896 rows in every launch of k_merge_long (one workgroup each, up
    to 256 at once), repeated: the same trace, counter and result as the oracle every time."""
    rng = np.random.default_rng(n + groups)
    rows = clustered(rng, n, 32, groups, noise)
    want = oracle.cluster(rows, 0.8, 3, 1000000, 17, 4)
    for _ in range(3):
        with options(engine, tail_merge_rows=1):
            engine.load_rows(rows)
            trace, counter, st = engine.cluster(0.8, 3, 1000000, 17, 4)
            got = engine.result()
        assert st["kern"]["huge"]["launches"] > 0
        assert np.array_equal(trace, want[3]) and counter == want[4]
        assert_same_result(got, *want[:3])


def test_long_runs_in_the_loop_vs_oracle(engine, oracle):
    """The cluster loop with buckets over 896 rows every iteration (few tight groups at d = 32):
    same N_t trace, counter and result as the oracle."""
    rng = np.random.default_rng(77)
    rows = clustered(rng, 30000, 32, 12, 0.03)
    want = oracle.cluster(rows, 0.8, 6, 1000000, 41, 4)
    with options(engine, tail_merge_rows=1):
        engine.load_rows(rows)
        trace, counter, st = engine.cluster(0.8, 6, 1000000, 41, 4)
        got = engine.result()
    assert st["kern"]["huge"]["launches"] > 0
    assert np.array_equal(trace, want[3]) and counter == want[4]
    assert_same_result(got, *want[:3])


@pytest.mark.parametrize("gram", [8, 32, 0])
def test_wide_gram_group_merges_vs_oracle(engine, oracle, gram):
    """C5-width (d = 512) group merges with their pairwise decisions from the bf16x3 Gram tile
    (option wide_gram, certified with the width's own margin) or from the exact chains: same
    trace, counter and result as the oracle, special rows (huge, tiny, zero, NaN) included."""
    rng = np.random.default_rng(512 + gram)
    rows = clustered(rng, 30000, 512, 900, 0.05)
    rows[5] *= np.float32(1e20)
    rows[11] *= np.float32(1e-20)
    rows[13] = 0.0
    rows[17, 2] = np.nan
    want = oracle.cluster(rows, 0.8, 4, 1000000, 31, 4)
    with options(engine, wide_gram=gram, tail_merge_rows=1):
        engine.load_rows(rows)
        trace, counter, _ = engine.cluster(0.8, 4, 1000000, 31, 4)
        got = engine.result()
    assert np.array_equal(trace, want[3]) and counter == want[4]
    assert_same_result(got, *want[:3])


@pytest.mark.parametrize("b", [2, 3, 5, 9, 17, 33, 64])
def test_small_screen_pcluster_special_rows(engine, oracle, b):
    """One small run through the screen (pcluster: the rows as one bucket) with a row the fp16
    image cannot carry: ADVICE r03 (a huge row must keep its run for the exact merge)."""
    rng = np.random.default_rng(b)
    for special in ("huge", "tiny", "zero", "nan", "none"):
        rows = clustered(rng, b, 64, max(1, b // 4), 0.02)
        k = b // 2
        if special == "huge":
            rows[k] *= np.float32(3e4)
        elif special == "tiny":
            rows[k] *= np.float32(1e-9)
        elif special == "zero":
            rows[k] = 0.0
        elif special == "nan":
            rows[k, 0] = np.nan
        with options(engine, small_screen=1, tail_merge_rows=1):
            engine.load_rows(rows)
            engine.pcluster(0.9)
            got = engine.result()
        assert_same_result(got, *oracle.pcluster(rows, 0.9)), (b, special)


@pytest.mark.parametrize("b", [17, 33, 64])
@pytest.mark.parametrize("gram", [8, 32])
def test_wide_gram_close_calls_vs_oracle(engine, oracle, b, gram):
    """d = 512 runs whose pairwise cosines crowd the threshold (rows = unit center + isotropic
    noise scaled so E[cos] = thr: about 1 % of the pairs fall inside the certified margin,
    wide_gram_margin(512) = 1.37e-4), so the Gram tiles' hit / miss masks AND their close-call
    path (gram_decide_slow, the exact chains) both decide pairs of one tile — the shape that broke
    a d = 512 parity test when round 5 tried reusing the masks for the close calls.  Special rows
    (huge, tiny, zero, NaN) in half of the runs; several runs per bucket-free pcluster call."""
    rng = np.random.default_rng(b * 31 + gram)
    d, thr = 512, 0.9
    s = np.sqrt((1.0 / thr - 1.0) / d)
    for rep in range(4):
        c = rng.normal(0, 1, size=d)
        c /= np.linalg.norm(c)
        rows = (c[None, :] + rng.normal(0, s, size=(b, d))).astype(np.float32)
        if rep & 1:
            rows[1] *= np.float32(1e20)
            rows[2] *= np.float32(1e-20)
            rows[3] = 0.0
            rows[4, 7] = np.nan
        with options(engine, wide_gram=gram, tail_merge_rows=1):
            engine.load_rows(rows)
            engine.pcluster(thr)
            got = engine.result()
        assert_same_result(got, *oracle.pcluster(rows, thr)), (b, gram, rep)


def seq_sim(a, c):
    """The reference's sim for one pair, op by op in fp32 (distance.cc:27-38)."""
    f = np.float32
    dot, na, nc = f(0), f(0), f(0)
    for u, v in zip(a, c):
        dot = f(dot + f(u * v))
        na = f(na + f(u * u))
        nc = f(nc + f(v * v))
    return f(dot / f(np.sqrt(na) * np.sqrt(nc)))


@pytest.mark.parametrize("b,d,step", [(40, 16, 0), (40, 16, 1), (40, 16, -1), (200, 64, 0),
                                      (200, 64, 1), (600, 8, 0), (3000, 8, 0)])
def test_pcluster_threshold_ties(engine, oracle, b, d, step):
    """Thresholds exactly at (step 0) or one ulp either side of a pair's similarity: the merge
    test's fast quotient bounds must hand these to the correctly rounded division."""
    rng = np.random.default_rng(b + d)
    rows = clustered(rng, b, d, max(2, b // 20), 0.08)
    f = np.float32
    for a, c in [(1, 0), (b // 2, b // 3), (b - 1, 2)]:
        sim = seq_sim(rows[a], rows[c])
        thr = f(f(1) - f(f(1) - sim))
        for _ in range(abs(step)):
            thr = np.nextafter(thr, f(np.inf if step > 0 else -np.inf), dtype=np.float32)
        engine.load_rows(rows)
        engine.pcluster(float(thr))
        assert_same_result(engine.result(), *oracle.pcluster(rows, float(thr)))


@pytest.mark.parametrize("b,d", [(33, 64), (1000, 16), (5000, 8)])
def test_pcluster_identical_rows(engine, oracle, b, d):
    """Degenerate bucket (every row identical): the wave kernel merges i into j = 0 each step."""
    rows = np.tile(np.linspace(-1, 2, d, dtype=np.float32), (b, 1))
    engine.load_rows(rows)
    engine.pcluster(0.95)
    assert_same_result(engine.result(), *oracle.pcluster(rows, 0.95))


# ------------------------------------------------------------------------------- Cluster ----
CLUSTER_CASES = ["cluster_d16", "cluster_d64", "cluster_d12", "cluster_d8_init", "cluster_nested",
                 "cluster_nested_small"]


@pytest.mark.parametrize("name", CLUSTER_CASES)
def test_cluster_matches_reference(engine, name):
    z = golden(name + ".npz")
    engine.load_rows(z["rows"])
    trace, counter, stats = engine.cluster(float(z["min_sim"]), int(z["iters"]), int(z["bthr"]),
                                           int(z["seed"]), 0)
    assert np.array_equal(trace, z["trace"])
    assert_same_result(engine.result(), z["out_rows"], z["out_off"], z["out_ids"])


def test_cluster_weighted_matches_reference(engine):
    z = golden("cluster_weighted.npz")
    engine.load_rows(z["rows"], z["in_off"], z["in_ids"])
    trace, _, _ = engine.cluster(float(z["min_sim"]), int(z["iters"]), int(z["bthr"]),
                                 int(z["seed"]), 0)
    assert np.array_equal(trace, z["trace"])
    assert_same_result(engine.result(), z["out_rows"], z["out_off"], z["out_ids"])


def test_convert_matches_reference(engine):
    z = golden("convert.npz")
    engine.load_counts(z["counts"], z["v_kmers"])
    rows, off, ids = engine.result()
    assert np.array_equal(ids, z["out_ids"])
    assert np.array_equal(np.diff(off), np.ones(len(ids), np.uint64))
    assert same_bits(rows, z["out_rows"])


def clustered(rng, n, d, groups, noise):
    centers = rng.normal(0, 1, size=(groups, d)).astype(np.float32)
    return (centers[rng.integers(0, groups, n)] +
            rng.normal(0, noise, size=(n, d)).astype(np.float32)).astype(np.float32)


@pytest.mark.parametrize("n,d,groups,iters,bthr", [
    (200000, 64, 4000, 12, 1000000),
    (100000, 32, 500, 8, 1000000),
    (60000, 20, 300, 6, 1000000),      # wide kernels, one partial chunk
    (30000, 512, 400, 5, 1000000),     # C5 width
    (50000, 16, 3, 3, 5000),           # nested path in every iteration
])
def test_cluster_random_vs_oracle(engine, oracle, n, d, groups, iters, bthr):
    rng = np.random.default_rng(n + d)
    rows = clustered(rng, n, d, groups, 0.05)
    engine.load_rows(rows)
    trace, counter, _ = engine.cluster(0.8, iters, bthr, 777, 3)
    o_rows, o_off, o_ids, o_trace, o_counter = oracle.cluster(rows, 0.8, iters, bthr, 777, 3)
    assert np.array_equal(trace, o_trace)
    assert counter == o_counter
    assert_same_result(engine.result(), o_rows, o_off, o_ids)


@pytest.mark.parametrize("n,d,groups,iters,bthr,long_runs", [
    (50000, 16, 3, 3, 5000, 4), (60000, 32, 20, 4, 1000000, 4), (60000, 32, 20, 4, 1000000, 1),
    (60000, 32, 20, 4, 1000000, 0), (50000, 16, 10, 3, 1000000, 0), (60000, 8, 20, 4, 1000000, 4),
    (60000, 64, 20, 4, 1000000, 4)])
def test_cluster_huge_fold_vs_oracle(engine, oracle, n, d, groups, iters, bthr, long_runs):
    """The loop with every >896-row run walked inside the 385..896-row kernel (option huge_fold),
    nested buckets included, through the per-class launches (tail_merge_rows = 1).  Where the fold
    is the path (every width but d = 16 / 32 with long_runs = 4, whose >384-row runs are
    k_merge_long's) no launch of the >896-row class is made although such runs exist: the fold
    walked them."""
    rng = np.random.default_rng(n + d + 1)
    rows = clustered(rng, n, d, groups, 0.05)
    with options(engine, huge_fold=1, tail_merge_rows=1, long_runs=long_runs):
        engine.load_rows(rows)
        trace, counter, st = engine.cluster(0.8, iters, bthr, 777, 3)
        got = engine.result()
    o_rows, o_off, o_ids, o_trace, o_counter = oracle.cluster(rows, 0.8, iters, bthr, 777, 3)
    assert np.array_equal(trace, o_trace) and counter == o_counter
    assert_same_result(got, o_rows, o_off, o_ids)
    huge = st["kern"]["huge"]
    assert huge["runs"] > 0  # runs over 896 rows were listed
    if d in (16, 32) and long_runs == 4:
        assert huge["launches"] > 0  # k_merge_long
    else:
        assert huge["launches"] == 0  # folded into the 385..896-row kernel


@pytest.mark.parametrize("window", [7, 40, 100])
def test_cluster_small_hyperplane_window_vs_oracle(engine, oracle, window):
    """Hyperplanes drawn in a bounded window (refilled when the loop reaches its end, also
    under the queued-ahead projection and nested buckets) give the oracle's result bit for bit."""
    rng = np.random.default_rng(window)
    rows = clustered(rng, 20000, 16, 300, 0.05)
    engine.load_rows(rows)
    engine.set_option("hyperplane_window", window)
    try:
        trace, counter, _ = engine.cluster(0.8, 40, 2000, 31, 5)
    finally:
        engine.set_option("hyperplane_window", 0)
    o_rows, o_off, o_ids, o_trace, o_counter = oracle.cluster(rows, 0.8, 40, 2000, 31, 5)
    assert np.array_equal(trace, o_trace)
    assert counter == o_counter
    assert_same_result(engine.result(), o_rows, o_off, o_ids)


@pytest.mark.parametrize("d,bthr,asy", [(13, 1000000, 1), (16, 2000, 1), (64, 1000000, 1),
                                         (16, 2000, 0)])
def test_cluster_hyperplane_async_vs_oracle(engine, oracle, d, bthr, asy):
    """Option hyperplane_async (default 1): the call's hyperplanes drawn by a background host
    thread while the first iterations run, uploaded as the loop needs them — d = 13 (padded rows
    of the window), nested buckets (bthr = 2000: their draws run past the predrawn window and
    fall back to the synchronous refill), twice in a row on one context (the drawer restarted)."""
    rng = np.random.default_rng(d + bthr)
    rows = clustered(rng, 30000, d, 400, 0.05)
    want = oracle.cluster(rows, 0.8, 30, bthr, 41, 7)
    with options(engine, hyperplane_async=asy):
        for _ in range(2):
            engine.load_rows(rows)
            trace, counter, _ = engine.cluster(0.8, 30, bthr, 41, 7)
            assert np.array_equal(trace, want[3]) and counter == want[4]
            assert_same_result(engine.result(), *want[:3])


def test_cluster_repeat_and_restore_deterministic(engine):
    rng = np.random.default_rng(5)
    rows = clustered(rng, 100000, 64, 2000, 0.05)
    engine.load_rows(rows)
    engine.snapshot()
    engine.cluster(0.8, 10, 1000000, 1, 0)
    a = engine.result()
    engine.restore()
    engine.cluster(0.8, 10, 1000000, 1, 0)
    b = engine.result()
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_empty_and_single(engine):
    engine.load_rows(np.zeros((0, 8), np.float32))
    trace, counter, _ = engine.cluster(0.8, 3, 10, 1, 0)
    assert list(trace) == [0, 0, 0] and counter == 0
    engine.load_rows(np.ones((1, 8), np.float32))
    trace, counter, _ = engine.cluster(0.8, 3, 10, 1, 0)
    assert list(trace) == [1, 1, 1] and counter == 0


# ------------------------------------------------------------------- mode C, end to end ------
@pytest.mark.parametrize("kat", ["katF", "katG", "katN"])
def test_cli_kat_md5(kat, tmp_path):
    import kat_inputs
    from kmerlsh_amd import _native

    with open(os.path.join(GOLDEN, "kat_md5.json")) as f:
        ref = json.load(f)[kat]
    kat_inputs.write_kat(kat, str(tmp_path))
    out = subprocess.run([_native.CLI_PATH, "-a", "a.txt", "-b", "b.txt", "-I", "10", "-M", "C",
                          "--only", "--seed", "12345", "--verbose"], cwd=tmp_path, check=True,
                         capture_output=True, text=True, timeout=300).stdout
    for fn, md5 in ref["md5"].items():
        with open(tmp_path / fn, "rb") as f:
            assert hashlib.md5(f.read()).hexdigest() == md5, fn
    trace = [int(line.split(":")[1]) for line in out.splitlines() if line.startswith("Size of")]
    assert trace == ref["trace"]


@pytest.mark.parametrize("thresh", [3000, 7000])
def test_cli_recluster_branch_vs_oracle(oracle, thresh, tmp_path):
    """init_clustering's multi-batch first pass and its `while (total > batch_thresh)` re-cluster
    passes (similarity -= 0.001, I + 4; app/kmerLSH.cc:303-411), reached on katF's 20K rows by the
    test-only KLSH_TEST_BATCH_THRESH override in both CLIs: the product's outputs equal the oracle
    CLI's byte for byte.  (Pinned product <-> oracle only: the reference hard-codes 1e8, and
    reaching the branch there needs > 1e8 k-mers.)"""
    import kat_inputs
    from kmerlsh_amd import _native

    outs = {}
    for name, cli in (("gpu", _native.CLI_PATH), ("oracle", oracle.CLI)):
        d = tmp_path / name
        kat_inputs.write_kat("katF", str(d))
        env = dict(os.environ, KLSH_TEST_BATCH_THRESH=str(thresh))
        out = subprocess.run([cli, "-a", "a.txt", "-b", "b.txt", "-I", "10", "-T", "2", "-M", "C",
                              "--only", "--seed", "12345", "--verbose"], cwd=d, check=True,
                             capture_output=True, text=True, timeout=300, env=env).stdout
        trace = [int(line.split(":")[1]) for line in out.splitlines() if line.startswith("Size of")]
        outs[name] = (trace, {fn: hashlib.md5(open(d / fn, "rb").read()).hexdigest()
                              for fn in ("clustering_result.txt", "clustering_result.txt.clust")})
    assert outs["gpu"] == outs["oracle"]
    # the branch ran: more than one init batch and at least one re-cluster pass
    assert len(outs["gpu"][0]) > 10 + 20000 // thresh


def test_synth_mode_c_vs_oracle(engine, oracle):
    """klsh-synth counts -> GPU convert -> init pass -> main loop, against the oracle."""
    from kmerlsh_amd import _native

    n, d = 400000, 32
    counts, cov = _native.synth_counts(n, d, seed=13)
    v_kmers = (cov.astype(np.float32) / np.float32(n)).astype(np.float32)
    engine.load_counts(counts, v_kmers)
    t0, c0, _ = engine.cluster(0.8, 1, 100000, 12345, 0)
    t1, c1, _ = engine.cluster(0.8, 10, 1000000, 12345, c0)
    got = engine.result()
    rows, ids = oracle.convert(counts, v_kmers)
    r1, o1, i1, tr0, k0 = oracle.cluster(rows, 0.8, 1, 100000, 12345, 0, None, ids)
    r2, o2, i2, tr1, k1 = oracle.cluster(r1, 0.8, 10, 1000000, 12345, k0, o1, i1)
    assert np.array_equal(t0, tr0) and np.array_equal(t1, tr1) and c1 == k1
    assert_same_result(got, r2, o2, i2)


def test_full_size_c2_properties(engine):
    """C2 shape (10M x 64) on random data: size-independent properties of the GPU result (the
    oracle is too slow at this size for every test run; the bench workload itself is pinned
    bit-exact over all 500 iterations by tests/test_gpu_fullsize.py and bench.py's post-check)."""
    from kmerlsh_amd import _native

    n, d = 10_000_000, 64
    counts, cov = _native.synth_counts(n, d, seed=11)
    v_kmers = (cov.astype(np.float32) / np.float32(n)).astype(np.float32)
    engine.load_counts(counts, v_kmers)
    del counts
    n_kept, _ = engine.count()
    _, c0, _ = engine.cluster(0.8, 1, 100000, 12345, 0)
    engine.snapshot()
    trace, c1, st = engine.cluster(0.8, 20, 1000000, 12345, c0)
    rows, off, ids = engine.result()
    assert np.all(np.diff(trace.astype(np.int64)) <= 0)          # N_t never grows
    assert int(off[-1]) == n_kept                                 # members partition the rows
    assert np.array_equal(np.sort(ids), np.unique(ids)) and ids.size == n_kept
    assert np.all(np.isfinite(rows))
    engine.restore()                                              # replay: identical
    trace2, c2, _ = engine.cluster(0.8, 20, 1000000, 12345, c0)
    rows2, off2, ids2 = engine.result()
    assert np.array_equal(trace, trace2) and c1 == c2
    assert np.array_equal(off, off2) and np.array_equal(ids, ids2) and same_bits(rows, rows2)


@pytest.mark.parametrize("b,d,groups,noise,thr,special", [
    (70, 64, 4, 0.05, 0.999, False), (70, 64, 4, 0.05, 0.9, False), (200, 64, 6, 0.08, 0.99, True),
    (384, 64, 3, 0.05, 0.995, True), (384, 64, 3, 0.05, 0.8, False), (130, 32, 5, 0.05, 0.995, True),
    (300, 32, 200, 0.3, 0.9, False), (128, 32, 2, 0.01, 0.9, True)])
@pytest.mark.parametrize("screen", [1, 0])
def test_tail_big_screen_vs_oracle(engine, oracle, b, d, groups, noise, thr, special, screen):
    """Option tail_big_screen (default 1): a 65..384-row run in k_merge_tail is screened on the fp16
    image first and left alone when no pair can pass — merge-free runs (thresholds close to 1),
    merge-dense runs, and rows the image cannot carry (fp16 overflow, all-zero image of a nonzero
    row, zero, NaN), with the screen on and off: the oracle's result bit for bit."""
    rng = np.random.default_rng(b * 13 + d + int(thr * 1000))
    rows = clustered(rng, b, d, groups, noise)
    if special:
        rows[5] *= np.float32(1e5)      # fp16 overflow in the image
        rows[9] *= np.float32(1e-9)     # image all zero
        rows[11] = 0.0
        rows[17, 3] = np.nan
    with options(engine, tail_big_screen=screen):
        engine.load_rows(rows)
        engine.pcluster(thr)
        got = engine.result()
    assert_same_result(got, *oracle.pcluster(rows, thr))


@pytest.mark.parametrize("d", [32, 64])
def test_cluster_tail_big_screen_vs_oracle(engine, oracle, d):
    """The loop through k_merge_tail with big runs (tight groups, thresholds stepping down from
    0.95): every iteration's 65..384-row runs screened on the fp16 image first."""
    rng = np.random.default_rng(d + 99)
    rows = clustered(rng, 120000, d, 600, 0.03)
    want = oracle.cluster(rows, 0.8, 10, 1000000, 17, 2)
    engine.load_rows(rows)
    trace, counter, st = engine.cluster(0.8, 10, 1000000, 17, 2)
    assert st["kern"]["tail"]["launches"] == 10
    assert sum(st["kern"][c]["runs"] for c in ("big128", "big192", "big384")) == 0  # all in the tail
    assert np.array_equal(trace, want[3]) and counter == want[4]
    assert_same_result(engine.result(), *want[:3])
