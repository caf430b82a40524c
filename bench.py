"""Benchmark: the kmerLSH main LSH+cluster loop on the gfx950 engine.

Metric (BASELINE.json): k-mers·iterations/s of the main Cluster() loop
(reference app/kmerLSH.cc:490, function/cluster.cc:181-340) = N_0 * I / T_loop.

Workload (BASELINE.json configs[1], "C2"): 10M k-mers x 64 samples, -I 500 -N 0.80.  Input is
klsh-synth v1 (seed 11), converted on the GPU (mode C, convertHTMat) and
put through the reference's init pass (one iteration at 0.95, bucket threshold 1e5) before timing;
the timed step is the main loop: restore the post-init state (device-to-device) and run all
500 iterations (bucket threshold 1e6).  Inputs are resident in HBM when timing starts.

Multi-GPU: one process per GPU (torch.distributed.run), BASELINE configs[2] ("C3"): the same
10M x 64 problem sharded across the ranks by key range with RCCL exchanges over
xGMI (keys/slots all-to-all, merge-delta allgather) and a result identical to 1 GPU: strong
scaling, value = N_0 * I / T of the one job.  --mode replicas instead runs an independent matrix
per rank (seed 11 + rank, no collective; weak scaling).  Barrier + max-over-ranks timing.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c2|c4|c5]
                    [--mode sharded|replicas] [--cpu-baseline auto|reference|port|full|none]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "k-mers·iterations/sec (LSH+cluster loop), 10M k-mers × 64 samples"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_TFLOPS = 78.6  # packed f32 mul / add issue ceiling (see roofline["valu"])

CONFIGS = {
    # name: (kmers, samples, iterations, min_similarity, synth seed, description)
    "c1": (100_000, 8, 10, 0.80, 1, "C1: 100K k-mers x 8 samples, -I 10 -N 0.80"),
    "c2": (10_000_000, 64, 500, 0.80, 11, "C2: 10M k-mers x 64 samples, -I 500 -N 0.80"),
    "c4": (100_000_000, 32, 100, 0.80, 13, "C4: 100M k-mers x 32 samples, -I 100 -N 0.80"),
    "c5": (10_000_000, 512, 500, 0.80, 17, "C5: 10M k-mers x 512 samples, -I 500 -N 0.80"),
}
SEED_BASE = 12345  # hyperplane seeding convention


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # host-side control only (timing scalars, the RCCL id); the data path runs over RCCL
        # inside the engine
        dist.init_process_group(backend="gloo", rank=rank, world_size=world)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(world, value: float) -> float:
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def device_sync(local: int) -> None:
    """torch.cuda.synchronize() (the engine already syncs its own stream before returning)."""
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.synchronize(local)


def timed(step, steps: int, warmup: int, world: int, local: int = 0, sync=device_sync):
    """W untimed steps, then exactly K steps bracketed by barrier + device sync on both sides;
    returns (max over ranks of the elapsed seconds, the K step results)."""
    for _ in range(warmup):
        step()
    sync(local)
    barrier(world)
    t0 = time.perf_counter()
    results = [step() for _ in range(steps)]
    sync(local)
    barrier(world)
    elapsed = time.perf_counter() - t0
    return max_over_ranks(world, elapsed), results


def prepare(eng, n, d, seed):
    """synth counts -> GPU convert -> init pass; returns (rng counter, kept rows, init stats)."""
    from kmerlsh_amd import _native
    from kmerlsh_amd.io import v_kmers_from_coverage

    t0 = time.time()
    counts, cov = _native.synth_counts(n, d, seed=seed)
    v_kmers = v_kmers_from_coverage(cov, n)  # as the reference reads kmer_count.log
    log(f"synth {n}x{d} in {time.time() - t0:.1f}s")
    eng.load_counts(counts, v_kmers)
    del counts
    kept, _ = eng.count()
    # init pass (app/kmerLSH.cc:323): one iteration at 0.95, bucket threshold 1e5
    _, counter, st0 = eng.cluster(0.80, 1, 100_000, SEED_BASE, 0)
    eng.snapshot()
    log(f"init pass: {kept} -> {st0['n_final']} rows ({st0['wall_ms']:.1f} ms)")
    return counter, kept, st0


def state_at(eng, t, min_sim, iters, counter0):
    """The loop's state at the start of iteration t (the engine stopped after t iterations)."""
    eng.restore()
    if t > 0:
        eng.set_option("stop_after", t)
        try:
            eng.cluster(min_sim, iters, 1_000_000, SEED_BASE, counter0)
        finally:
            eng.set_option("stop_after", 0)
    return eng.result()


def schedule_threshold(min_sim, iters, t):
    """Cluster()'s threshold at iteration t (function/cluster.cc:190-192,330), in float32 as the
    reference computes it: 0.95f, then -= sim_step per iteration."""
    thr = np.float32(0.95)
    step = np.float32((np.float32(0.95) - np.float32(min_sim)) / np.float32(iters))
    for _ in range(t):
        thr = np.float32(thr - step)
    return float(thr)


def write_state(tmp, rows, off, ids):
    src = os.path.join(tmp, "rows.f32")
    rows.astype("<f4").tofile(src)
    off.astype("<u8").tofile(src + ".off")
    ids.astype("<u8").tofile(src + ".ids")
    return src


def cpu_baseline(eng, mode, n0, d, iters, min_sim, counter0, trace):
    """The reference (oracle/_ref/ref_harness: the reference's own functions, compiled from its
    sources) or the oracle port, timed on this host's cores.

    Default (a bounded sample): 3 consecutive iterations of the loop from its own state at 10
    points t in [0, .9 I] (the engine provides the state) at the schedule's thresholds — the
    harness's iter_w, Cluster()'s loop body through the reference's p_lsh, merge_hashtable,
    p_cluster / nestedCluster and merge_abundance (Cluster() itself would start at 0.95) — the
    2nd and 3rd timed.  Their per-row cost, interpolated in t and weighted by the loop's N_t
    trace, estimates T_loop; value
    = N_0 * I / T_loop like the metric.  mode "full": the reference's WHOLE main loop timed once
    (its own Cluster() over all I iterations from the post-init state, ~5 min at C2 on 16
    threads), with the sampled estimate beside it."""
    if mode == "none":
        return None
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    threads = min(16, os.cpu_count() or 1)
    kind = None
    if mode in ("auto", "reference", "full") and os.path.exists(harness):
        kind = "reference"
    elif mode in ("auto", "port"):
        kind = "port"
    if kind is None:
        return None
    env = dict(os.environ, OMP_THREAD_LIMIT=str(threads), OMP_NUM_THREADS=str(threads),
               KLSH_REF_THREADS=str(threads), KLSH_SEED=str(SEED_BASE))
    full = None
    if mode == "full" and kind == "reference":
        rows, off, ids = state_at(eng, 0, min_sim, iters, counter0)
        n_t = rows.shape[0]
        with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
            src = write_state(tmp, rows, off, ids)
            del rows, off, ids
            log(f"cpu baseline: the reference's whole loop, {iters} iterations from {n_t} rows, "
                f"{threads} threads")
            # (its verbose output streamed: a progress line every 25 iterations keeps a long run
            # visibly alive)
            proc = subprocess.Popen([harness, "cluster_w", src, src + ".off", src + ".ids",
                                     str(n_t), str(d), repr(float(min_sim)), str(iters), "1000000",
                                     os.path.join(tmp, "out")], env=env, stdout=subprocess.PIPE,
                                    text=True)
            lines = []
            for ln in proc.stdout:
                lines.append(ln)
                if ln.startswith("Iteration:"):
                    it = int(ln.split()[1].rstrip(","))
                    if it % 25 == 0:
                        log(f"cpu baseline: reference iteration {it}/{iters}")
            if proc.wait(timeout=3000) != 0:
                raise RuntimeError(f"ref_harness cluster_w exited with {proc.returncode}")
            out = "".join(lines)
        secs = float(re.findall(r"hash\+cluster takes \(secs\): ([0-9.eE+-]+)", out)[-1])
        sizes = [int(v) for v in re.findall(r"Size of profilings\D*(\d+)", out)]
        log(f"cpu baseline: reference loop {secs:.1f} s")
        # (at T > 1 the reference's concatenation order depends on OpenMP scheduling,
        # cluster.cc:281, so its N_t trace is its own, not the T = 1 trace the engine matches)
        full = {"value": n0 * iters / secs, "loop_s": secs, "sum_trace": int(sum(sizes[-iters:])),
                "final_rows": int(re.findall(r"after clustering:\s*(\d+)", out)[-1])}
    trace = np.asarray(trace, dtype=np.float64)
    # 10 windows, densest where N_t and the per-row cost change fastest (the head).  Each runs 3
    # consecutive iterations of the loop from the state at t and times the 2nd and 3rd: those run
    # on the state the reference's own loop left (its allocations, grown member lists), which on
    # the box costs ~1.4x a state freshly built from arrays (the first iteration of a window).
    ts = sorted({min(iters - 3, int(f * iters))
                 for f in (0.0, 0.05, 0.1, 0.15, 0.2, 0.3, 0.4, 0.5, 0.7, 0.9)})
    step = np.float32((np.float32(0.95) - np.float32(min_sim)) / np.float32(iters))
    cost, at, secs_all = [], [], 0.0
    for t in ts:
        rows, off, ids = state_at(eng, t, min_sim, iters, counter0)
        n_t = rows.shape[0]
        thr_t = schedule_threshold(min_sim, iters, t)
        if kind == "reference":
            with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
                src = write_state(tmp, rows, off, ids)
                del rows, off, ids
                out = subprocess.run([harness, "iter_w", src, src + ".off", src + ".ids",
                                      str(n_t), str(d), repr(thr_t), "1000000", "3",
                                      repr(float(step))], env=env,
                                     check=True, capture_output=True, text=True,
                                     timeout=900).stdout
            it_s = [float(v) for v in re.findall(r"one iteration takes \(secs\): ([0-9.eE+-]+)", out)]
            it_n = [int(v) for v in re.findall(r"iteration: (\d+) ->", out)]
            for j in (1, 2):
                cost.append(it_s[j] / max(1, it_n[j]))
                at.append(t + j)
            secs_all += sum(it_s)
            log(f"cpu baseline ({kind}, {threads} threads): t={t}..{t + 2} N_t={n_t}: "
                + " / ".join(f"{v:.2f}" for v in it_s) + " s")
            continue
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import klsh_oracle

        t0 = time.perf_counter()  # (the oracle's one-iteration call runs at 0.95)
        klsh_oracle.cluster(rows, float(min_sim), 1, 1_000_000, SEED_BASE, 0, off, ids, threads)
        secs = time.perf_counter() - t0
        log(f"cpu baseline ({kind}, {threads} threads): t={t} N_t={n_t}: {secs:.2f} s")
        secs_all += secs
        cost.append(secs / max(1, n_t))
        at.append(t)
    per_row = np.interp(np.arange(len(trace)), at, cost)
    t_loop = float((trace * per_row).sum())
    c1 = c1_measured(harness) if kind == "reference" else None
    sampled = {"value": n0 * iters / t_loop, "estimated_loop_s": round(t_loop, 2),
               "sample_seconds": round(secs_all, 2),
               "sample": ((f"3 consecutive iterations of the main loop from its own state at t = "
                           f"{', '.join(map(str, ts))} of {iters} ({threads} threads, the "
                           f"schedule's thresholds, reference harness iter_w), the 2nd and 3rd "
                           f"timed" if kind == "reference" else
                           f"one iteration from the state at t = {', '.join(map(str, ts))} of "
                           f"{iters} (the port's one-iteration call runs at 0.95)") +
                          f"; per-row cost interpolated in t and weighted by the loop's N_t "
                          f"trace (sum N_t = {int(trace.sum())}) to estimate T_loop")}
    if full:
        return {"value": full["value"], "unit": "k-mers·iterations/s", "cores": threads,
                "kind": "reference_full", "loop_s": round(full["loop_s"], 2),
                "reference_sum_trace": full["sum_trace"], "reference_final_rows": full["final_rows"],
                "sample": (f"the reference's whole main loop ({iters} iterations, its own Cluster()"
                           f" through oracle/_ref/ref_harness cluster_w) from the post-init state, "
                           f"{threads} threads, timed once"),
                "sampled_estimate": dict(sampled, ratio_to_full=round(t_loop / full["loop_s"], 4)),
                "c1_measured": c1}
    out = dict({"unit": "k-mers·iterations/s", "cores": threads, "kind": kind, "c1_measured": c1},
               **sampled)
    # the reference's whole loop as measured once on a GPU box's host (bench.py --cpu-baseline
    # full, committed in profiles/cpu_reference_full.json), beside this run's sampled estimate
    committed = reference_full_committed(n0, d, iters)
    if committed:
        committed["ratio_sampled_to_full"] = round(t_loop / committed["loop_s"], 4)
        out["reference_full"] = committed
    return out


def reference_full_committed(n0, d, iters):
    """The committed whole-loop measurement of the reference for this workload (C2 only)."""
    path = os.path.join(ROOT, "profiles", "cpu_reference_full.json")
    if (n0, d, iters) != (10_000_000, 64, 500) or not os.path.exists(path):
        return None
    with open(path) as f:
        rec = dict(json.load(f)["c2"])
    rec["value"] = n0 * iters / rec["loop_s"]
    rec["unit"] = "k-mers·iterations/s"
    return rec


def c1_measured(harness, threads=1):
    """The reference's WHOLE main loop on C1 (BASELINE configs[0]: 100K x 8, -I 10 -N 0.80, "1
    thread CPU OpenMP reference"), timed at OMP_THREAD_LIMIT=1 -T 1 as that config states: the C1
    workload through the engine's convert + init pass (GPU), then the reference's own Cluster()
    (ref_harness) over all 10 iterations from that state, and the engine's loop on the same state
    for comparison.  A measured full loop beside C2's sampled estimate."""
    from kmerlsh_amd import _native

    n0, d, iters, min_sim, seed, _ = CONFIGS["c1"]
    eng = _native.Engine(0)
    try:
        counter0, kept, _ = prepare(eng, n0, d, seed)
        rows, off, ids = eng.result()
        n_t = rows.shape[0]
        with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
            src = os.path.join(tmp, "rows.f32")
            rows.astype("<f4").tofile(src)
            off.astype("<u8").tofile(src + ".off")
            ids.astype("<u8").tofile(src + ".ids")
            env = dict(os.environ, OMP_THREAD_LIMIT=str(threads), OMP_NUM_THREADS=str(threads),
                       KLSH_REF_THREADS=str(threads), KLSH_SEED=str(SEED_BASE))
            out = subprocess.run([harness, "cluster_w", src, src + ".off", src + ".ids", str(n_t),
                                  str(d), repr(float(min_sim)), str(iters), "1000000",
                                  os.path.join(tmp, "out")], env=env, check=True,
                                 capture_output=True, text=True, timeout=600).stdout
        secs = float(re.findall(r"hash\+cluster takes \(secs\): ([0-9.eE+-]+)", out)[-1])
        eng.restore()
        t0 = time.perf_counter()
        eng.cluster(min_sim, iters, 1_000_000, SEED_BASE, counter0)
        gpu = time.perf_counter() - t0
    finally:
        eng.close()
    log(f"C1 full loop: reference {secs:.3f} s ({threads} threads), engine {gpu * 1e3:.2f} ms")
    return {"loop_s": secs, "value": n0 * iters / secs, "unit": "k-mers·iterations/s",
            "cores": threads, "rows_after_init": int(n_t),
            "engine_loop_ms": round(gpu * 1e3, 3), "engine_value": n0 * iters / gpu,
            "note": "C1 (100K x 8, -I 10): the reference's whole main loop timed (ref_harness), "
                    "from the engine's post-init state; engine timed on the same state"}


def check_parity(config, trace, counter, result):
    """Compare the last timed step with the committed full-size fixture (tests/golden/
    fullsize_<config>.json: the oracle's — for C1/C2 also the reference CLI's — run of the same
    workload).  Full loops: trace, rng counter and result md5s; pinned prefixes: the trace."""
    import hashlib

    path = os.path.join(ROOT, "tests", "golden", f"fullsize_{config}.json")
    if not os.path.exists(path):
        return {"checked": False}
    with open(path) as f:
        fx = json.load(f)
    k = fx["run_iterations"]
    out = {"checked": True, "fixture": os.path.relpath(path, ROOT), "iterations_pinned": k,
           "trace": [int(v) for v in trace[:k]] == fx["trace"]}
    if k == fx["iterations"]:
        rows, off, ids = result()
        md5 = lambda a: hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa: E731
        out["counter"] = counter == fx["counter"]
        out["md5"] = (md5(rows) == fx["md5_rows"] and md5(off) == fx["md5_offsets"] and
                      md5(ids) == fx["md5_ids"])
    out["ok"] = all(v for key, v in out.items() if key in ("trace", "counter", "md5"))
    return out


def pmc_traffic(config, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        data = json.load(f)
    return (data.get(config) or {}).get(kernel)


# Algorithmic bytes of one kernel class over a step, from the class's own row
# counters (klsh_stats.kern: rows handled, runs) — what the class must move at minimum:
#   project   rows x (4d row + 4 slot + 4 key)
#   sort      sum over iterations of N_t x passes_t x 20 (hist: key; scatter: key + slot in and out)
#   runs      rows x 4 (sorted keys) + runs x 8 (list entries)
#   small     rows x (4d + 4) (row + slot) + merges x (4d + 20) (new row, norm, count, head, link);
#             after the screen, its rows are those of the runs the screen passed
#   screen    rows x (2d + 4) (fp16 row + slot) + runs x 8 (list entries)
#   big*/huge rows x (4d + 20) (row, slot, count, head, tail, the slot written back)
#   tail      rows x (4d + 8) (all merge classes of a small iteration in one launch)
#   compact   rows x 12 (slots read twice, survivors written)
KERNEL_NAMES = {
    "project": "k_project_pk<{d}>", "sort": "k_sort_hist/dscan/scatter (span)",
    "runs": "k_runs_count/scan/write (span)", "small": "k_merge_small<{d}>",
    "big128": "k_merge_big<{d},128,128,true>", "big192": "k_merge_big<{d},192,256,true>",
    "big384": "k_merge_big<{d},384,256,true>", "big896": "k_merge_big<{d},896,256,false>",
    "huge": "k_merge_huge<{d}>", "tail": "k_merge_tail<{d}>",
    "compact": "k_compact_count/apply (span)", "screen": "k_small_screen<{d}>",
}
WIDE_NAMES = {
    "project": "k_project_mfma_wide + k_project_fix (span)",
    "small": "k_merge_group_wide<64..2> (six launches on four streams, span)",
    "big128": "k_merge_big_wide<128,128,32>", "big192": "k_merge_big_wide<384,256,32>",
    "big384": "k_merge_big_wide<384,256,32>", "big896": "k_merge_big_wide<896,256,16>",
    "huge": "k_merge_huge<0>",
}
BF16_DENSE_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)


def kernel_rooflines(config, stats, steps, d, trace, shadow, tail_rows=1 << 22):
    """Every kernel class's achieved HBM rate (its algorithmic bytes per launch over its average
    HIP-event launch time); the headline is the class with the largest time per step."""
    register = d in (8, 16, 32, 64)
    # SURVEY.md 8(d) bytes: the projection reads the f32 row (4d), a slot and writes a key.
    # shadow: what it actually reads is the fp16 row image (2d bytes a row; the engine keeps one at
    # d = 16, 32, 64 unless option "projection" = 1),
    # plus the f32 row of the close calls: reported beside it as "image"
    row_bytes = 4 * d
    kern = {c: {f: sum(s["kern"][c][f] for s in stats) for f in ("ms", "launches", "rows", "runs")}
            for c in stats[0]["kern"]}
    merge_phase = kern.pop("merge", None)
    merges_small = sum(s["small_iter_merges"] for s in stats)
    tr = np.asarray(trace, dtype=np.float64)
    tr = tr[tr > 1]
    passes = np.ceil(np.floor(np.log2(tr)) / 10.0) if tr.size else tr
    sort_bytes = float((tr * passes * 20.0).sum()) * steps
    out = []
    for c, k in kern.items():
        if not k["launches"] or k["ms"] <= 0:
            continue
        rows, runs = k["rows"], k["runs"]
        b = {"project": rows * (row_bytes + 8), "sort": sort_bytes, "runs": rows * 4 + runs * 8,
             "screen": rows * (2 * d + 4) + runs * 8,
             "small": rows * (4 * d + 4) + merges_small * (4 * d + 20),
             "tail": rows * (4 * d + 8), "compact": rows * 12}.get(c, rows * (4 * d + 20))
        avg = k["ms"] / k["launches"]
        ach = (b / k["launches"]) / (avg * 1e-3) / 1e9
        name = (KERNEL_NAMES if register or c not in WIDE_NAMES else WIDE_NAMES)[c].format(d=d)
        if c == "project" and shadow:
            name = f"k_project_h16<{d}>"
        if c == "huge" and d in (16, 32):
            name = f"k_merge_long<{d}>"
        pmc = pmc_traffic(config, c) or pmc_traffic(config, {"project": "k_project",
                                                             "small": "k_merge_small",
                                                             "screen": "k_small_screen"}.get(c, ""))
        e = {"kernel": name, "class": c, "bound": "hbm", "achieved": round(ach, 2),
             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5),
             "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
             "traffic_source": (pmc or {}).get("source"),
             "bytes_per_launch": b / k["launches"], "avg_launch_ms": avg,
             "launches_per_step": k["launches"] / steps, "ms_per_step": k["ms"] / steps,
             "rows_per_launch": rows / k["launches"]}
        # the same launches through HIP events on their own stream, where that measures the
        # kernel (the projection and the small-run launch run alone on theirs; a big-run class
        # shares the CUs with them and an event pair would include its waits for resources)
        ev_ms = {"project": sum(s["project_ms"] for s in stats),
                 "small": sum(s["small_ms"] for s in stats)}.get(c)
        ev_n = {"project": sum(s["project_timed_launches"] for s in stats),
                "small": sum(s["small_launches"] for s in stats)}.get(c)
        e["timing"] = "stamps"
        if ev_ms and ev_n:
            e["hip_events"] = {"avg_launch_ms": ev_ms / ev_n, "launches_per_step": ev_n / steps,
                               "ms_per_step": ev_ms / steps}
            if ev_n == k["launches"]:
                # the HIP-event time of the same launches is the reported rate; stamps beside it
                ev_avg = ev_ms / ev_n
                ach_ev = (b / k["launches"]) / (ev_avg * 1e-3) / 1e9
                e["stamps"] = {"achieved": e["achieved"], "frac": e["frac"], "avg_launch_ms": avg}
                e["stamps"]["ms_per_step"] = e["ms_per_step"]
                e.update(achieved=round(ach_ev, 2), frac=round(ach_ev / HBM_PEAK_GBS, 5),
                         avg_launch_ms=ev_avg, ms_per_step=ev_ms / steps, timing="hip_events")
        if c == "project":
            bits = sum(s["sum_proj_bits"] for s in stats)
            if shadow:
                # The headline rate is on the bytes this kernel must move: it reads the fp16 row
                # image (2d) + a slot and writes a key per row.  SURVEY.md 8(d)'s figure (the f32
                # row, 4d + 8) is the same launch time over bytes the kernel does not read: kept
                # beside it as "survey_8d_equivalent", never as the achieved rate.
                ib = rows * (2 * d + 8) / k["launches"]
                ia = ib / (e["avg_launch_ms"] * 1e-3) / 1e9
                e["survey_8d_equivalent"] = {
                    "bytes_per_launch": e["bytes_per_launch"], "achieved": e["achieved"],
                    "frac": e["frac"],
                    "note": "SURVEY.md 8(d) bytes (f32 row 4d + slot + key per row) over the same "
                            "launch time: a normalized rate, not traffic (the kernel reads the "
                            "fp16 image instead of the f32 row)"}
                e.update(bytes_per_launch=ib, achieved=round(ia, 2),
                         frac=round(ia / HBM_PEAK_GBS, 5),
                         bytes_note="fp16 row image (2d) + slot + key per row: the bytes the "
                                    "kernel must move; close calls re-read their f32 row on top "
                                    "(in traffic)")
                if "stamps" in e:
                    sa = ib / (e["stamps"]["avg_launch_ms"] * 1e-3) / 1e9
                    e["stamps"].update(achieved=round(sa, 2), frac=round(sa / HBM_PEAK_GBS, 5))
                # the fp16-image screen: S = X~ (w_hi + w_lo)^T, 2 f16 MFMA products per product
                # (wide rows: a third, |x~|.|w_hi|, for the bound)
                fl = (2 if register else 3) * 2.0 * bits * d / k["launches"]
                e["mfma"] = {"achieved": round(fl / (avg * 1e-3) / 1e12, 2),
                             "peak": BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                             "note": "fp16 row image x w split into fp16 hi + lo on "
                                     "v_mfma_f32_32x32x16_f16 (2 products per product, dense f16 "
                                     "peak); close calls settled in the kernel on the f32 row"}
                e["mfma"]["frac"] = round(e["mfma"]["achieved"] / BF16_DENSE_TFLOPS, 5)
                fixed = sum(s.get("proj_fix_pairs", 0) for s in stats)
                e["close_calls"] = {"pairs": fixed / steps, "frac_of_pairs": fixed / max(1, bits),
                                    "note": "row-hyperplane pairs per step the screen left to the "
                                            "exact f32 chains"}
            elif register:
                # one v_pk_mul + one v_pk_add per two row-hyperplane MACs (bit-exactness forbids
                # fusing): 256 CU x 4 SIMD x 32 lanes x 2 flop x 2.4 GHz / 2 = 78.6 Tflop/s
                fl = 2.0 * bits * d / k["launches"]
                e["valu"] = {"achieved": round(fl / (avg * 1e-3) / 1e12, 2), "peak": VALU_PEAK_TFLOPS,
                             "unit": "TFLOP/s", "note": "separate f32 mul + add (no FMA: bit-exact "
                                                        "with the reference), packed v_pk_mul/v_pk_add"}
                e["valu"]["frac"] = round(e["valu"]["achieved"] / VALU_PEAK_TFLOPS, 4)
            else:
                # the certified screen: S = X W^T as fp16x3 (hi.hi + hi.lo + lo.hi) plus the
                # |x|.|w| bound product, 4 f16 MFMA products per f32 product, against the dense
                # f16 peak; the exact fix-up of the close calls is in the span too
                fl = 4 * 2.0 * bits * d / k["launches"]
                e["mfma"] = {"achieved": round(fl / (avg * 1e-3) / 1e12, 2),
                             "peak": BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                             "note": "fp16x3 split + |x|.|w| bound on v_mfma_f32_32x32x16_f16 (4 "
                                     "products per f32 product); span includes k_project_fix"}
                e["mfma"]["frac"] = round(e["mfma"]["achieved"] / BF16_DENSE_TFLOPS, 5)
                fixed = sum(s.get("proj_fix_pairs", 0) for s in stats)
                e["close_calls"] = {"pairs": fixed / steps, "frac_of_pairs": fixed / max(1, bits),
                                    "note": "row-hyperplane pairs per step k_project_fix settled "
                                            "with the exact f32 chains"}
        out.append(e)
    if not out:
        return {}
    # The merge classes of an iteration run concurrently on four streams: a
    # class's stamp span then includes its waits for CUs behind the others, so it is not that
    # kernel's own launch time.  The headline is the kernel with the largest time per step among
    # the launches that run alone (projection, sort, runs, the one-launch tail merge,
    # compaction); the concurrent classes stay listed with "overlapped": true.
    for e in out:
        if e["class"] in ("big128", "big192", "big384", "big896", "huge", "small", "screen"):
            e["overlapped"] = True
    alone = [e for e in out if not e.get("overlapped")] or out
    head = dict(max(alone, key=lambda e: e["ms_per_step"]))
    head["kernels"] = sorted(out, key=lambda e: -e["ms_per_step"])
    # The merge PHASE of the iterations whose classes run as separate concurrent launches
    # (N_t >= tail_rows, the engine's "tail_merge_rows", at the register widths; every iteration
    # at d > 64): first workgroup start of any
    # merge class to the last end, per iteration (KLSH_K_MERGE stamps), against SURVEY.md 8(d)'s
    # merge share of B_t: N_t x 4d (every row read for the in-bucket merge) + M_t x (4d + 8) (the
    # new row and a member link per merge), summed over those iterations.
    if merge_phase and merge_phase["launches"]:
        tr = np.asarray(trace, dtype=np.float64)
        nxt = np.append(tr[1:], float(stats[-1]["n_final"]))
        sel = tr >= tail_rows if register else tr >= 0
        mb = float((tr[sel] * 4 * d + (tr[sel] - nxt[sel]) * (4 * d + 8)).sum())
        ms = merge_phase["ms"] / steps
        n_it = merge_phase["launches"] / steps
        ach = mb / (ms * 1e-3) / 1e9
        head["phases"] = [{
            "phase": "merge wall of the multi-launch iterations" +
                     (f" (N_t >= {tail_rows})" if register else ""),
            "iterations_per_step": n_it, "ms_per_step": ms, "bytes_per_step": mb,
            "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 5),
            "note": "KLSH_K_MERGE stamps: per iteration, the first merge-class workgroup start to "
                    "the last end (the concurrent small-run screen, small-run merge and big-run "
                    "classes together); bytes SURVEY.md 8(d): N_t*4d + M_t*(4d+8) over those "
                    "iterations of the last step's trace"}]
    head["note"] = ("roofline = the kernel class with the largest time per step among the launches "
                    "that run alone (the concurrent merge classes are marked overlapped: their spans "
                    "include waits for CUs behind each other); a launch's time "
                    "is its first workgroup start -> last workgroup end from in-kernel "
                    "s_memrealtime stamps (rocprofv3's kernel span), hip_events = the HIP event "
                    "pair on the launch's own stream where that isolates it; 'span' classes cover "
                    "several dependent launches")
    return head


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-baseline", default="auto",
                    choices=["auto", "reference", "port", "full", "none"],
                    help="full: the reference's whole main loop timed once (C2: minutes)")
    ap.add_argument("--mode", default="sharded", choices=["sharded", "replicas"],
                    help="N>1: one problem sharded over the ranks (C3) or one problem per rank")
    ap.add_argument("--phases", action="store_true",
                    help="per-phase HIP-event timing (sort/merge/compaction); adds latency")
    ap.add_argument("--shard1", action="store_true",
                    help="profiling only: run the sharded loop on one GPU (in-process group of 1)")
    ap.add_argument("--iterations", type=int, default=0,
                    help="profiling only: override the config's -I (the metric is then not C2's)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="engine option (klsh_set_option), e.g. small_screen=1; repeatable")
    args = ap.parse_args()

    world, rank, local = dist_setup()
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}")
    n0, d, iters, min_sim, synth_seed, desc = CONFIGS[args.config]
    if args.iterations:
        iters = args.iterations
        desc += f" [profiling override: -I {iters}]"
    from kmerlsh_amd import _native

    eng = _native.Engine(local)
    if args.phases:
        eng.set_option("phase_timing", 1)
    for opt in args.option:
        name, _, val = opt.partition("=")
        eng.set_option(name, int(val))
    sharded = world > 1 and args.mode == "sharded"
    if sharded:
        import torch.distributed as dist

        uid = [_native.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(rank, world, uid[0])
        log(f"rank {rank}/{world}: RCCL group up")
    elif args.shard1:
        _native.comm_init_local([eng])
    counter0, kept, _ = prepare(eng, n0, d, seed=synth_seed if sharded else synth_seed + rank)

    def step():
        eng.restore()
        return eng.cluster(min_sim, iters, 1_000_000, SEED_BASE, counter0)

    elapsed, results = timed(step, args.steps, args.warmup, world, local)
    log(f"{args.steps} timed steps: {elapsed:.3f} s (max over {world} ranks)")
    stats = [r[2] for r in results]
    trace, counter = results[-1][0], results[-1][1]

    if rank != 0:
        return
    # outside the timed region: the last step's output against the committed full-size fixture
    parity = (check_parity(args.config, trace, counter, eng.result)
              if (world == 1 or sharded) and not args.iterations else {"checked": False})
    if parity.get("checked"):
        log(f"parity vs {parity['fixture']}: {'ok' if parity['ok'] else 'MISMATCH'}")
    value = (1 if sharded else world) * n0 * iters * args.steps / elapsed
    agg = {k: sum(s[k] for s in stats) for k in stats[0] if k != "kern"}
    phases = {p: agg[p + "_ms"] / args.steps
              for p in ("project", "sort", "merge", "compact", "host", "comm", "small")}
    for c in ("runs", "tail", "compact"):
        phases[c] = sum(s["kern"][c]["ms"] for s in stats) / args.steps
    # Kernel rooflines.  The projection: algorithmic bytes per launch = rows x
    # (4d row + 4 slot + 4 key).  The small-run merge (runs of 2..64 rows; its own launch in the
    # iterations of >= tail_merge_rows positions, timed by HIP events on its stream):
    # rows x (4d row + 4 slot) + merges x (4d new row + 20 metadata: norm, count, head, member
    # link, the removed row's count) — merges counted over the whole iteration (~97 % of them are
    # small-run merges on C2).  The bench line's "roofline" is the one with the larger time per step.
    roofline = kernel_rooflines(args.config, stats, args.steps, d, trace,
                                bool(eng.get_option("fp16_image")) and d <= 64,
                                eng.get_option("tail_merge_rows"))
    # the whole loop against HBM, SURVEY.md §8(d): B_t = N_t (8d + 16) + M_t (4d + 8) bytes per
    # iteration (rows read by the projection and by the merge, keys and order written and read;
    # per merge the new row and a member link), summed over the timed steps
    loop_bytes = agg["sum_rows"] * (8 * d + 16) + agg["sum_merges"] * (4 * d + 8)
    loop_gbs = loop_bytes / elapsed / 1e9
    roofline["loop"] = {"achieved": round(loop_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(loop_gbs / HBM_PEAK_GBS, 5),
                        "bytes_per_step": loop_bytes / args.steps,
                        "note": "SURVEY.md 8(d) algorithmic bytes of the whole loop / step time"}
    cpu = None
    if world == 1:
        try:
            cpu = cpu_baseline(eng, args.cpu_baseline, n0, d, iters, min_sim, counter0, trace)
        except Exception as e:  # the baseline is reported, never required
            log(f"cpu baseline failed: {e}")
    line = {
        "metric": METRIC if args.config == "c2" else f"k-mers·iterations/sec, {desc}",
        "value": value,
        "unit": "k-mers·iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1000.0,
        "higher_is_better": True,
        # the default mode keeps the C2 problem fixed as N grows (N = 1 included, so the driver's
        # N = 1, 2, 4, 8 lines describe one series); --mode replicas gives every rank its own
        "scaling": "strong" if args.mode == "sharded" else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": (f"synthetic klsh-synth v1 (seed {synth_seed}), {kept} rows kept of {n0}"
                 if world == 1 or sharded else
                 f"synthetic klsh-synth v1 (seed {synth_seed}+rank), {kept} rows kept of {n0} per rank"),
        "config": {"workload": desc + " (main Cluster loop after the init pass)", "kmers": n0,
                   "samples": d, "iterations": iters, "min_similarity": min_sim,
                   "bucket_size_threshold": 1_000_000,
                   "parallelism": (f"sharded x{world} (key ranges, RCCL)" if sharded else
                                   f"replicas x{world}" if world > 1 else "single GPU")},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "phases_ms_per_step": phases,
        "rows_projected_per_step": agg["sum_rows"] / args.steps,
        "final_clusters": stats[-1]["n_final"],
        "nested_calls_per_step": agg["nested_calls"] / args.steps,
        "parity": parity,
    }
    if args.option:
        line["options"] = args.option
    print(json.dumps(line), flush=True)
    if parity.get("checked") and not parity["ok"]:
        sys.exit(1)  # a fast wrong answer is not a result


if __name__ == "__main__":
    main()
