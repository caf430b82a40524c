"""The sharded multi-GPU loop against the single-GPU engine and the reference.

RCCL refuses two ranks on one device, so the sharded path is exercised here through the
in-process group (klsh_comm_init_local): W contexts on the one GPU, each driven by its own host
thread, exchanging through the same Comm interface RCCL implements.  Everything but the
transport is the product code path.  Bar: bit-exact — N_t trace, rng counter, survivor order,
member lists and centroid bits equal the single-GPU call (and the reference's goldens).
"""
import threading

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a, np.float32).view(np.uint32),
                          np.ascontiguousarray(b, np.float32).view(np.uint32))


def run_group(world, load, calls, shard_min_rows=0):
    """Create `world` engines on device 0, load each with load(eng), bind them into one group,
    run the klsh_cluster calls (list of argument tuples) on every rank concurrently.  Returns
    per-rank lists of (trace, counter, stats) and the per-rank results.  shard_min_rows = 0
    keeps every iteration sharded; larger values switch to the replicated tail below it."""
    from kmerlsh_amd import _native

    engines = [_native.Engine(0) for _ in range(world)]
    try:
        for e in engines:
            load(e)
            e.set_option("shard_min_rows", shard_min_rows)
        _native.comm_init_local(engines)
        for r, e in enumerate(engines):
            assert e.comm_info() == (r, world)
        outs = [None] * world
        errs = []

        def work(r):
            try:
                res = []
                counter = None
                for (ms, it, bthr, seed, c0) in calls:
                    c = c0 if counter is None or c0 is not None else counter
                    trace, counter, st = engines[r].cluster(ms, it, bthr, seed, c)
                    res.append((trace, counter, st))
                outs[r] = res
            except Exception as ex:  # surfaced below
                errs.append((r, ex))

        ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=600)
        assert not any(t.is_alive() for t in ts), "sharded call hung"
        assert not errs, errs
        results = [e.result() for e in engines]
        return outs, results
    finally:
        for e in engines:
            e.close()


def single(engine, load, calls):
    load(engine)
    res = []
    counter = None
    for (ms, it, bthr, seed, c0) in calls:
        c = c0 if counter is None or c0 is not None else counter
        trace, counter, st = engine.cluster(ms, it, bthr, seed, c)
        res.append((trace, counter, st))
    return res, engine.result()


def assert_same(a_res, a_out, b_res, b_out):
    for (ta, ca, _), (tb, cb, _) in zip(a_res, b_res):
        assert np.array_equal(ta, tb)
        assert ca == cb
    ra, oa, ia = a_out
    rb, ob, ib = b_out
    assert np.array_equal(oa, ob)
    assert np.array_equal(ia, ib)
    assert same_bits(ra, rb)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["cluster_d16", "cluster_d64", "cluster_d12", "cluster_nested",
                                  "cluster_nested_small"])
def test_sharded_matches_reference(world, name):
    z = golden(name + ".npz")
    calls = [(float(z["min_sim"]), int(z["iters"]), int(z["bthr"]), int(z["seed"]), 0)]
    outs, results = run_group(world, lambda e: e.load_rows(z["rows"]), calls)
    for r in range(world):
        trace, _, st = outs[r][0]
        assert st["world"] == world
        assert np.array_equal(trace, z["trace"]), r
        rows, off, ids = results[r]
        assert np.array_equal(off, z["out_off"]) and np.array_equal(ids, z["out_ids"]), r
        assert same_bits(rows, z["out_rows"]), r


def test_sharded_weighted_matches_reference():
    z = golden("cluster_weighted.npz")
    calls = [(float(z["min_sim"]), int(z["iters"]), int(z["bthr"]), int(z["seed"]), 0)]
    outs, results = run_group(2, lambda e: e.load_rows(z["rows"], z["in_off"], z["in_ids"]), calls)
    for r in range(2):
        assert np.array_equal(outs[r][0][0], z["trace"])
        rows, off, ids = results[r]
        assert np.array_equal(off, z["out_off"]) and np.array_equal(ids, z["out_ids"])
        assert same_bits(rows, z["out_rows"])


def clustered(rng, n, d, groups, noise):
    centers = rng.normal(0, 1, size=(groups, d)).astype(np.float32)
    return (centers[rng.integers(0, groups, n)] +
            rng.normal(0, noise, size=(n, d)).astype(np.float32)).astype(np.float32)


@pytest.mark.parametrize("world,n,d,groups,iters,bthr", [
    (2, 200000, 64, 4000, 12, 1000000),
    (4, 200000, 64, 4000, 12, 1000000),
    (3, 100000, 32, 500, 8, 1000000),
    (2, 60000, 20, 300, 6, 1000000),     # generic kernels
    (4, 50000, 16, 3, 3, 5000),          # nested buckets on several ranks every iteration
    (8, 3000, 8, 40, 6, 1000000),        # more ranks than some key ranges have rows
])
def test_sharded_random_vs_single(engine, world, n, d, groups, iters, bthr):
    rng = np.random.default_rng(n + d + world)
    rows = clustered(rng, n, d, groups, 0.05)
    calls = [(0.8, iters, bthr, 777, 3)]
    ref = single(engine, lambda e: e.load_rows(rows), calls)
    outs, results = run_group(world, lambda e: e.load_rows(rows), calls)
    for r in range(world):
        assert_same(outs[r], results[r], *ref)


@pytest.mark.parametrize("world,switch", [(2, 150000), (3, 120000), (4, 1 << 19)])
def test_sharded_then_replicated_tail_vs_single(engine, world, switch):
    """The crossover: sharded while N_t >= switch, then every rank runs the rest on its replica."""
    rng = np.random.default_rng(world * 7 + 1)
    rows = clustered(rng, 200000, 64, 30000, 0.05)
    calls = [(0.8, 15, 1000000, 777, 3)]
    ref = single(engine, lambda e: e.load_rows(rows), calls)
    assert ref[0][0][0][0] >= switch or switch > 200000  # the run starts sharded unless above n
    outs, results = run_group(world, lambda e: e.load_rows(rows), calls, shard_min_rows=switch)
    for r in range(world):
        assert_same(outs[r], results[r], *ref)


def test_sharded_mode_c_two_calls_vs_single(engine):
    """Init pass + main loop (two calls carrying the rng counter), mode-C rows from synth."""
    from kmerlsh_amd import _native

    n, d = 300000, 64
    counts, cov = _native.synth_counts(n, d, seed=21)
    v_kmers = (cov.astype(np.float32) / np.float32(n)).astype(np.float32)
    calls = [(0.8, 1, 100000, 12345, 0), (0.8, 25, 1000000, 12345, None)]
    ref = single(engine, lambda e: e.load_counts(counts, v_kmers), calls)
    outs, results = run_group(2, lambda e: e.load_counts(counts, v_kmers), calls)
    for r in range(2):
        assert_same(outs[r], results[r], *ref)


def test_sharded_empty_and_single_row():
    calls = [(0.8, 3, 10, 1, 0)]
    outs, _ = run_group(2, lambda e: e.load_rows(np.zeros((0, 8), np.float32)), calls)
    assert [list(o[0][0]) for o in outs] == [[0, 0, 0]] * 2
    outs, res = run_group(3, lambda e: e.load_rows(np.ones((1, 8), np.float32)), calls)
    assert [list(o[0][0]) for o in outs] == [[1, 1, 1]] * 3
    assert all(r[0].shape == (1, 8) for r in res)


def test_rccl_single_rank_group_vs_single(engine):
    """The RCCL backend itself (a one-rank communicator: its allgather, broadcast-based
    allgather-v, all-to-all self copy and min all-reduce) driving the sharded loop."""
    from kmerlsh_amd import _native

    rng = np.random.default_rng(11)
    rows = clustered(rng, 100000, 64, 2000, 0.05)
    calls = [(0.8, 10, 1000000, 5, 0)]
    ref = single(engine, lambda e: e.load_rows(rows), calls)
    eng = _native.Engine(0)
    try:
        eng.load_rows(rows)
        eng.comm_init(0, 1, _native.comm_unique_id())
        eng.set_option("shard_min_rows", 0)
        trace, counter, st = eng.cluster(*calls[0])
        assert st["world"] == 1 and st["comm_ms"] > 0.0
        assert_same([(trace, counter, st)], eng.result(), *ref)
    finally:
        eng.close()


def test_sharded_failure_aborts_the_group():
    """A rank that fails (here: nothing loaded) aborts the group: the other rank's collectives
    return an error instead of waiting for it forever, and the group stays unusable."""
    from kmerlsh_amd import _native

    rng = np.random.default_rng(5)
    rows = clustered(rng, 20000, 16, 500, 0.05)
    engines = [_native.Engine(0) for _ in range(2)]
    try:
        engines[0].load_rows(rows)
        for e in engines:
            e.set_option("shard_min_rows", 0)
        _native.comm_init_local(engines)
        errs = [None, None]

        def work(r):
            try:
                engines[r].cluster(0.8, 5, 1000000, 3, 0)
            except _native.KlshError as ex:
                errs[r] = str(ex)

        ts = [threading.Thread(target=work, args=(r,)) for r in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in ts), "a rank hung after its peer failed"
        assert errs[1] and "before a load" in errs[1]
        assert errs[0] and "abort" in errs[0]
        with pytest.raises(_native.KlshError, match="aborted"):
            engines[0].cluster(0.8, 5, 1000000, 3, 0)
    finally:
        for e in engines:
            e.close()
