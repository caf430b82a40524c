"""One rank of the CPU model of the sharded Cluster() loop, over gloo.

Run by tests/test_shard_model.py under torch.distributed.run.  The model follows the engine's
decomposition step by step — my block of the canonical order, keys of my clusters, the global
histogram of the top <= 12 key bits, bin ownership by row midpoint (k_bin_split's formula), the
stable exchange of clusters to their key range's owner (received in source-rank order), a stable
sort by key, p_cluster per bucket, the survivors as the next "mine" — with the oracle's hash and
p_cluster as the arithmetic.  The concatenation over ranks of the final "mine" must equal the
oracle's single-process Cluster() bit for bit.  TEST INFRASTRUCTURE: uses oracle/ as the checker.
"""
import json
import math
import os
import sys

import numpy as np
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import klsh_oracle as O  # noqa: E402

MAX_BIN_BITS = 12  # klsh_internal.h kMaxBinBits


def owners(hist, world):
    """k_bin_split (klsh_shard.hip): a bin goes to the rank its row midpoint falls in."""
    total = int(hist.sum())
    run = np.concatenate([[0], np.cumsum(hist, dtype=np.uint64)[:-1]]).astype(np.uint64)
    mid2 = 2 * run + hist.astype(np.uint64)
    if total == 0:
        return np.zeros(hist.size, dtype=np.int64)
    o = (mid2 * np.uint64(world)) // np.uint64(2 * total)
    return np.minimum(o.astype(np.int64), world - 1)


def main():
    dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    cfg = json.loads(os.environ["KLSH_MODEL_CFG"])
    rng = np.random.default_rng(cfg["seed"])
    n, d, iters, min_sim = cfg["n"], cfg["d"], cfg["iters"], cfg["min_sim"]
    centers = rng.normal(0, 1, (max(n // 20, 1), d)).astype(np.float32)
    rows = (centers[rng.integers(0, centers.shape[0], n)] +
            rng.normal(0, cfg["noise"], (n, d))).astype(np.float32)
    # clusters of the canonical order: (row, member ids); rank g owns block g
    lo, hi = n * rank // world, n * (rank + 1) // world
    mine = [(rows[i].copy(), [i]) for i in range(lo, hi)]

    max_sim = np.float32(0.95)  # cluster.cc:190-192, all float
    step = np.float32((max_sim - np.float32(min_sim)) / np.float32(iters))
    thr = max_sim
    counter = 0
    for _ in range(iters):
        cnt = [None] * world
        dist.all_gather_object(cnt, len(mine))
        N = sum(cnt)
        h = int(math.floor(math.log2(N))) if N > 0 else 0
        w, counter = O.table(cfg["rng_seed"], counter, h, d)
        keys = O.keys(np.array([c[0] for c in mine], np.float32).reshape(-1, d), w) if mine \
            else np.zeros(0, np.uint32)
        B = min(h, MAX_BIN_BITS)
        shift = h - B
        hist = np.bincount((keys >> shift).astype(np.int64), minlength=1 << B).astype(np.uint64)
        allh = [None] * world
        dist.all_gather_object(allh, hist)
        own = owners(np.sum(allh, axis=0), world)
        dest = own[(keys >> shift).astype(np.int64)] if mine else np.zeros(0, np.int64)
        parts = [[(int(keys[i]), mine[i]) for i in range(len(mine)) if dest[i] == r]
                 for r in range(world)]
        got = [None] * world
        dist.all_gather_object(got, parts)
        recv = [kc for src in range(world) for kc in got[src][rank]]  # source-rank order
        order = np.argsort(np.array([k for k, _ in recv], np.uint32), kind="stable")
        recv = [recv[i] for i in order]
        nxt = []
        a = 0
        while a < len(recv):
            b = a + 1
            while b < len(recv) and recv[b][0] == recv[a][0]:
                b += 1
            bucket = [c for _, c in recv[a:b]]
            if len(bucket) == 1:
                nxt.append(bucket[0])
            else:
                br = np.array([c[0] for c in bucket], np.float32)
                off = np.zeros(len(bucket) + 1, np.uint64)
                off[1:] = np.cumsum([len(c[1]) for c in bucket])
                ids = np.array([i for c in bucket for i in c[1]], np.uint64)
                out, oo, oi = O.pcluster(br, float(thr), off, ids)
                for j in range(out.shape[0]):
                    nxt.append((out[j].copy(), [int(v) for v in oi[int(oo[j]):int(oo[j + 1])]]))
            a = b
        mine = nxt
        thr = np.float32(thr - step)
    final = [None] * world
    dist.all_gather_object(final, mine)
    if rank == 0:
        allc = [c for r in range(world) for c in final[r]]
        out = {
            "rows": np.array([c[0] for c in allc], np.float32).view(np.uint32).tolist(),
            "ids": [c[1] for c in allc],
            "counter": counter,
        }
        with open(os.environ["KLSH_MODEL_OUT"], "w") as f:
            json.dump(out, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
