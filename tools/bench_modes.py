"""Throughput of the mode-E k-mer vote and the mode-B table build on one GPU (synthetic data).

  python tools/bench_modes.py [--reads 2000000] [--kset 4000000] [--samples 8] [--kmers 4000000]

Mode E: a FASTQ of random 150-bp reads, a third of them drawn from the sequence the k-mer set
was cut from, through klsh_extract_fastq (host parse + GPU vote + writer); reports reads/s, k-mer
probes/s of the vote kernel (HIP events) and the host parse time.
Mode B: `samples` KMC1 databases of `kmers` random 31-mers each (half shared), through
klsh_build_khtable; reports records/s.  Prints one JSON line per mode.
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def canonical_np(codes: np.ndarray, k: int) -> np.ndarray:
    """Canonical 8-byte images of every k-mer window of a code array (uint64)."""
    npos = codes.size - k + 1
    fwd = np.zeros(npos, np.uint64)
    rc = np.zeros(npos, np.uint64)
    for i in range(k):
        c = codes[i:i + npos].astype(np.uint64)
        fwd |= c << np.uint64(2 * i)
        rc |= (np.uint64(3) - c) << np.uint64(2 * (k - 1 - i))
    return np.where(fwd.byteswap() < rc.byteswap(), fwd, rc)


def bench_extract(engine, n_reads: int, n_kset: int, k: int = 31, vote: float = 0.5) -> dict:
    from kmerlsh_amd import _native

    rng = np.random.default_rng(3)
    src = rng.integers(0, 4, size=n_kset + k, dtype=np.uint8)
    kset = np.unique(canonical_np(src, k))
    L = 150
    starts = rng.integers(0, src.size - L, size=n_reads)
    rand = rng.integers(0, 4, size=(n_reads, L), dtype=np.uint8)
    from_src = (np.arange(n_reads) % 3) == 0
    idx = starts[from_src, None] + np.arange(L)[None, :]
    rand[from_src] = src[idx]
    seq = np.frombuffer(b"ACGT", np.uint8)[rand]
    qual = np.full((n_reads, L), ord("I"), np.uint8)
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
        path = os.path.join(tmp, "reads.fq")
        with open(path, "wb") as f:
            for a in range(0, n_reads, 100000):
                b = min(n_reads, a + 100000)
                recs = [b"@r%d\n%s\n+\n%s\n" % (i, seq[i].tobytes(), qual[i].tobytes()) for i in range(a, b)]
                f.write(b"".join(recs))
        ks = _native.KmerSet(engine, kset)
        ks.extract_fastq(path, os.path.join(tmp, "warm.fq"), k, vote)  # warm-up (page cache, code)
        t = time.perf_counter()
        st = ks.extract_fastq(path, os.path.join(tmp, "out.fq"), k, vote)
        wall = time.perf_counter() - t
        ks.close()
    probes = st["kmers_checked"]
    return {"mode": "E", "metric": "reads/s (k-mer vote + FASTQ parse + write)",
            "value": n_reads / wall, "reads": n_reads, "kset": int(kset.size), "k": k,
            "kernel_ms": st["kernel_ms"], "parse_ms": st["parse_ms"], "total_ms": st["total_ms"],
            "kernel_probes_per_s": probes / (st["kernel_ms"] / 1e3) if st["kernel_ms"] else None,
            "kernel_bytes_per_s": (st["bases"] + 8 * probes) / (st["kernel_ms"] / 1e3) if st["kernel_ms"] else None,
            "reads_extracted": st["reads_extracted"]}


def write_kmc1(path: str, k: int, values: np.ndarray, counts: np.ndarray, p: int = 11) -> None:
    """KMC1 layout (kmc_file.cpp:244-300) from sorted k-mer values (s[0] most significant)."""
    order = np.argsort(values, kind="stable")
    values, counts = values[order], counts[order]
    suf_sym = k - p
    pre = (values >> np.uint64(2 * suf_sym)).astype(np.int64)
    lut = np.zeros(1 << (2 * p), np.uint64)
    lut[1:] = np.cumsum(np.bincount(pre, minlength=1 << (2 * p)))[:-1]
    ss = suf_sym // 4
    suf = values & np.uint64((1 << (2 * suf_sym)) - 1)
    rec = np.zeros((values.size, ss + 2), np.uint8)
    for b in range(ss):
        rec[:, b] = ((suf >> np.uint64(8 * (ss - 1 - b))) & np.uint64(0xFF)).astype(np.uint8)
    rec[:, ss] = counts & 0xFF
    rec[:, ss + 1] = counts >> 8
    with open(path + ".kmc_suf", "wb") as f:
        f.write(b"KMCS" + rec.tobytes() + b"KMCS")
    hdr = struct.pack("<5Q", k, 2 | (p << 32), 1 | (65535 << 32), values.size, 0)
    with open(path + ".kmc_pre", "wb") as f:
        f.write(b"KMCP" + lut.tobytes() + hdr + struct.pack("<I", len(hdr)) + b"KMCP")


def bench_khtable(engine, samples: int, n_kmers: int, k: int = 31) -> dict:
    rng = np.random.default_rng(5)
    shared = rng.integers(0, 1 << (2 * k), size=n_kmers // 2, dtype=np.uint64)
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
        names = []
        for j in range(samples):
            own = rng.integers(0, 1 << (2 * k), size=n_kmers - shared.size, dtype=np.uint64)
            vals = np.unique(np.concatenate([shared, own]))
            cnts = rng.integers(1, 1000, size=vals.size).astype(np.uint16)
            name = os.path.join(tmp, "db%d" % j)
            write_kmc1(name, k, vals, cnts)
            names.append(name)
        engine.build_khtable(names[:1], k, tmp)  # warm-up
        t = time.perf_counter()
        st = engine.build_khtable(names, k, tmp)
        wall = time.perf_counter() - t
    return {"mode": "B", "metric": "KMC records/s (two passes: union, counts)",
            "value": st["records"] / wall, "samples": samples, "records": st["records"],
            "kmap_size": st["kmap_size"], "io_ms": st["io_ms"], "total_ms": st["total_ms"]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=2000000)
    ap.add_argument("--kset", type=int, default=4000000)
    ap.add_argument("--samples", type=int, default=8)
    ap.add_argument("--kmers", type=int, default=4000000)
    a = ap.parse_args()
    from kmerlsh_amd import _native

    with _native.Engine(0) as eng:
        print(json.dumps(bench_extract(eng, a.reads, a.kset)), flush=True)
        print(json.dumps(bench_khtable(eng, a.samples, a.kmers)), flush=True)


if __name__ == "__main__":
    main()
