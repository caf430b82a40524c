"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs oracle/_ref/ref_harness and oracle/_ref/kmerLSH_seeded (unmodified reference objects built
from /root/reference by `make -C oracle ref`, seeded per SURVEY.md §8(c), OMP_THREAD_LIMIT=1) on
small seeded inputs and stores inputs + the reference's outputs as .npz / .json data.
Needs /root/reference (this container only); the fixtures it writes are committed.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
REF_CLI = os.path.join(ROOT, "oracle", "_ref", "kmerLSH_seeded")
sys.path.insert(0, HERE)
import kat_inputs  # noqa: E402

ENV = dict(os.environ, OMP_THREAD_LIMIT="1", OMP_NUM_THREADS="1")


def run(args, seed=12345, cwd=None):
    env = dict(ENV, KLSH_SEED=str(seed))
    return subprocess.run(args, env=env, cwd=cwd, check=True, capture_output=True, text=True).stdout


def parse_clust(path):
    offs, ids = [0], []
    with open(path) as f:
        for line in f:
            parts = line.split()
            n = int(parts[0])
            ids.extend(int(v) for v in parts[1: 1 + n])
            offs.append(len(ids))
    return np.array(offs, dtype=np.uint64), np.array(ids, dtype=np.uint64)


def main_trace(stdout):
    """'Size of profilings' lines of the main loop (nested calls print them after
    '1-iter clustering')."""
    out, in_main = [], False
    for line in stdout.splitlines():
        if line.startswith("Iteration:"):
            in_main = True
        elif line.startswith("1-iter clustering"):
            in_main = False
        elif line.startswith("Size of profilings") and in_main:
            out.append(int(line.split(":")[1]))
            in_main = False
    return np.array(out, dtype=np.uint64)


def clustered_rows(rng, n, d, groups, noise, scale=1.0, order="random"):
    centers = rng.normal(0, scale, size=(groups, d)).astype(np.float32)
    g = rng.integers(0, groups, size=n)
    rows = centers[g] + rng.normal(0, noise, size=(n, d)).astype(np.float32)
    return rows.astype(np.float32)


def harness_cluster(tmp, rows, min_sim, iters, bthr, seed, weights=None):
    n, d = rows.shape
    prefix = os.path.join(tmp, "out")
    if weights is None:
        src = os.path.join(tmp, "rows.f32")
        rows.astype("<f4").tofile(src)
        so = run([HARNESS, "cluster", src, str(n), str(d), repr(float(min_sim)), str(iters),
                  str(bthr), prefix], seed)
    else:
        off, ids = weights
        src = os.path.join(tmp, "in.bin")
        rows.astype("<f4").tofile(src)
        with open(src + ".clust", "w") as f:
            for i in range(n):
                a, b = int(off[i]), int(off[i + 1])
                f.write(str(b - a) + "".join("\t%d" % v for v in ids[a:b]) + "\n")
        so = run([HARNESS, "cluster_from", src, str(d), repr(float(min_sim)), str(iters),
                  str(bthr), prefix], seed)
    out_rows = np.fromfile(prefix, dtype="<f4").reshape(-1, d)
    off, ids = parse_clust(prefix + ".clust")
    return out_rows, off, ids, main_trace(so)


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the reference first: make -C oracle ref")
    rng = np.random.default_rng(20261015)
    meta = {}
    with tempfile.TemporaryDirectory() as tmp:
        # 1. RNG known answers: generateHashTable(h, d) for several seeds.
        tables = {}
        for seed, h, d in [(12345, 3, 8), (1, 4, 16), (4294967295, 2, 64), (777, 23, 64),
                           (99, 5, 13)]:
            txt = run([HARNESS, "rng", str(h), str(d)], seed)
            w = np.array([[int(x, 16) for x in line.split()] for line in txt.strip().splitlines()],
                         dtype=np.uint32).view(np.float32)
            tables[f"s{seed}_h{h}_d{d}"] = w
        np.savez_compressed(os.path.join(HERE, "rng_tables.npz"), **tables)

        # 2. keys: LSH::random_projection over random rows, plus exact-zero / sign edge rows.
        for name, (n, d, h, seed) in {"keys_d8": (600, 8, 16, 5), "keys_d16": (600, 16, 12, 6),
                                      "keys_d64": (600, 64, 23, 7), "keys_d13": (600, 13, 9, 8),
                                      "keys_d512": (200, 512, 20, 9)}.items():
            rows = rng.normal(0, 1, size=(n, d)).astype(np.float32)
            rows[0] = 0.0                       # all-zero row: every sum is +0 -> all bits 1
            rows[1] = -0.0
            rows[2, :] = np.float32(1e-30)      # subnormal products
            rows[3, :] = np.float32(3e38)       # overflow to +-inf in the sum
            src = os.path.join(tmp, "k.f32")
            rows.astype("<f4").tofile(src)
            outp = os.path.join(tmp, "k.u32")
            run([HARNESS, "keys", src, str(n), str(d), str(h), outp], seed)
            keys = np.fromfile(outp, dtype="<u4")
            np.savez_compressed(os.path.join(HERE, name + ".npz"), rows=rows, keys=keys,
                                seed=np.uint32(seed), h=np.int32(h))

        # 3. p_cluster on single buckets (lane path <= 32, wave path > 32, generic d).
        for name, (b, d, groups, noise, thr) in {
            "pcluster_small": (24, 16, 4, 0.05, 0.95),
            "pcluster_large": (300, 64, 10, 0.08, 0.9),
            "pcluster_generic": (80, 12, 6, 0.1, 0.85),
            "pcluster_d8": (200, 8, 5, 0.15, 0.8),
        }.items():
            rows = clustered_rows(rng, b, d, groups, noise)
            src = os.path.join(tmp, "p.f32")
            rows.astype("<f4").tofile(src)
            prefix = os.path.join(tmp, "p")
            run([HARNESS, "pcluster", src, str(b), str(d), repr(float(np.float32(thr))), prefix])
            out_rows = np.fromfile(prefix, dtype="<f4").reshape(-1, d)
            off, ids = parse_clust(prefix + ".clust")
            np.savez_compressed(os.path.join(HERE, name + ".npz"), rows=rows,
                                thr=np.float32(thr), out_rows=out_rows, out_off=off, out_ids=ids)

        # 4. Cluster(): whole loop, traces and outputs.
        cases = {
            "cluster_d16": dict(n=5000, d=16, groups=120, noise=0.06, min_sim=0.8, iters=10,
                                bthr=1000000, seed=12345),
            "cluster_d64": dict(n=3000, d=64, groups=60, noise=0.05, min_sim=0.8, iters=8,
                                bthr=1000000, seed=4242),
            "cluster_d12": dict(n=2500, d=12, groups=80, noise=0.08, min_sim=0.7, iters=6,
                                bthr=1000000, seed=7),
            "cluster_d8_init": dict(n=4000, d=8, groups=50, noise=0.1, min_sim=0.8, iters=1,
                                    bthr=100000, seed=31337),
            "cluster_nested": dict(n=3000, d=8, groups=3, noise=0.0, min_sim=0.8, iters=3,
                                   bthr=200, seed=555),
            "cluster_nested_small": dict(n=600, d=16, groups=4, noise=0.02, min_sim=0.8, iters=4,
                                         bthr=20, seed=556),
        }
        for name, c in cases.items():
            rows = clustered_rows(rng, c["n"], c["d"], c["groups"], c["noise"])
            out_rows, off, ids, trace = harness_cluster(tmp, rows, c["min_sim"], c["iters"],
                                                        c["bthr"], c["seed"])
            np.savez_compressed(os.path.join(HERE, name + ".npz"), rows=rows,
                                min_sim=np.float32(c["min_sim"]), iters=np.int32(c["iters"]),
                                bthr=np.int32(c["bthr"]), seed=np.uint32(c["seed"]),
                                out_rows=out_rows, out_off=off, out_ids=ids, trace=trace)
            meta[name] = {k: (float(v) if isinstance(v, float) else v) for k, v in c.items()}

        # 5. weighted input (member lists of several ids, via ReadClusterAll).
        n, d = 1500, 16
        rows = clustered_rows(rng, n, d, 40, 0.05)
        sizes = rng.integers(1, 6, size=n)
        off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
        ids = rng.permutation(int(off[-1]) * 3)[: int(off[-1])].astype(np.uint64)
        out_rows, o2, i2, trace = harness_cluster(tmp, rows, 0.8, 6, 1000000, 2024,
                                                  weights=(off, ids))
        np.savez_compressed(os.path.join(HERE, "cluster_weighted.npz"), rows=rows, in_off=off,
                            in_ids=ids, min_sim=np.float32(0.8), iters=np.int32(6),
                            bthr=np.int32(1000000), seed=np.uint32(2024), out_rows=out_rows,
                            out_off=o2, out_ids=i2, trace=trace)

        # 6. mode-C producer (convertHTMat).
        n, d = 3000, 8
        counts = rng.poisson(3.0, size=(d, n)).astype(np.uint16)
        counts[:, :50] = 0                       # dropped rows (sum <= 0.1 d)
        counts[0, 50:60] = 65535                 # saturated counts
        v_kmers = (rng.random(d) * 2).astype(np.float32)
        src = os.path.join(tmp, "c.u16")
        counts.astype("<u2").tofile(src)
        vsrc = os.path.join(tmp, "v.f32")
        v_kmers.astype("<f4").tofile(vsrc)
        prefix = os.path.join(tmp, "cv")
        run([HARNESS, "convert", src, str(n), str(d), vsrc, prefix])
        out_rows = np.fromfile(prefix, dtype="<f4").reshape(-1, d)
        o3, i3 = parse_clust(prefix + ".clust")
        np.savez_compressed(os.path.join(HERE, "convert.npz"), counts=counts, v_kmers=v_kmers,
                            out_rows=out_rows, out_ids=i3)

        # 7. end-to-end mode-C KATs through the seeded reference CLI.
        kat = {}
        for k in ("katF", "katG", "katN"):
            wd = os.path.join(tmp, k)
            kat_inputs.write_kat(k, wd)
            so = run([REF_CLI, "-a", "a.txt", "-b", "b.txt", "-o", "A", "-p", "B", "-I", "10",
                      "-K", "23", "-T", "1", "-M", "C", "--only", "--verbose"], 12345, cwd=wd)
            md5 = {}
            for fn in ("kmer_count.bin", "kmer_count.log", "clustering_result.txt",
                       "clustering_result.txt.clust"):
                with open(os.path.join(wd, fn), "rb") as f:
                    md5[fn] = hashlib.md5(f.read()).hexdigest()
            kat[k] = {"md5": md5, "trace": main_trace(so).tolist(), "iters": 10, "seed": 12345}
        with open(os.path.join(HERE, "kat_md5.json"), "w") as f:
            json.dump(kat, f, indent=1, sort_keys=True)
    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
