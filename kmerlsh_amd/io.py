"""Mode-C file formats of the reference (byte-compatible readers/writers, host side).

  kmer_count.bin   sample-major uint16 LE, d columns of kmap_size   (io/ioHT.cc:59-81 ReadHT)
  kmer_count.log   "<kmap_size>\\t<coverage_1>...\\t<coverage_d>"    (app/kmerLSH.cc:471-482)
  <F>.clust        "<n>\\t<id>\\t...\\n" per cluster, n > ignore_small (io/ioMatrix.cc:265-294)
  <F>              raw fp32 rows of the same clusters, d per row      (io/ioMatrix.cc:322-351)
"""
from __future__ import annotations

import numpy as np


def count_lines(path: str) -> int:
    """Lines as std::getline counts them (io/ioHT.cc:3-19 GetInput)."""
    with open(path, "rb") as f:
        data = f.read()
    if not data:
        return 0
    return data.count(b"\n") + (0 if data.endswith(b"\n") else 1)


def read_count_log(path: str, d: int) -> tuple[int, np.ndarray]:
    """(kmap_size, v_kmers) with v_kmers[j] = float(coverage_j) / float(kmap_size)."""
    with open(path) as f:
        parts = f.read().split()
    kmap = int(parts[0])
    cov = np.array([np.float32(p) for p in parts[1: 1 + d]], dtype=np.float32)
    return kmap, (cov / np.float32(kmap)).astype(np.float32)


def v_kmers_from_coverage(coverage, kmap_size: int) -> np.ndarray:
    """v_kmers[j] exactly as the reference derives it from kmer_count.log: the coverage is
    written with "%f" (io/ioHT.cc:185), read back as float and divided by kmap_size in
    float (app/kmerLSH.cc:471-482)."""
    cov = np.array([np.float32(float("%f" % c)) for c in coverage], dtype=np.float32)
    return (cov / np.float32(kmap_size)).astype(np.float32)


def write_count_files(directory: str, counts: np.ndarray, coverage: np.ndarray) -> None:
    """kmer_count.bin/.log + a.txt/b.txt (d/2 samples each) for a (d, n) count matrix."""
    import os

    d, n = counts.shape
    counts.astype("<u2").tofile(os.path.join(directory, "kmer_count.bin"))
    with open(os.path.join(directory, "kmer_count.log"), "w") as f:
        f.write("%d" % n + "".join("\t%f" % c for c in coverage))
    with open(os.path.join(directory, "a.txt"), "w") as f:
        f.write("".join("s%d.fq k%d\n" % (j, j) for j in range(d // 2)))
    with open(os.path.join(directory, "b.txt"), "w") as f:
        f.write("".join("s%d.fq k%d\n" % (j, j) for j in range(d // 2, d)))


def save_result(path: str, member_offsets: np.ndarray, member_ids: np.ndarray,
                ignore_small: int = 5) -> None:
    with open(path, "wb") as f:
        for i in range(len(member_offsets) - 1):
            a, b = int(member_offsets[i]), int(member_offsets[i + 1])
            if b - a > ignore_small:
                f.write((str(b - a) + "".join("\t%d" % v for v in member_ids[a:b].tolist()) + "\n").encode())


def save_binary(path: str, rows: np.ndarray, member_offsets: np.ndarray,
                ignore_small: int = 5) -> None:
    sizes = np.diff(member_offsets.astype(np.int64))
    rows[sizes > ignore_small].astype("<f4").tofile(path)


def read_cluster_all(path: str, d: int):
    """io/ioMatrix.cc:48-119: rows from <path>, id lists from <path>.clust."""
    rows = np.fromfile(path, dtype="<f4").reshape(-1, d)
    offs = [0]
    ids: list[int] = []
    with open(path + ".clust") as f:
        for line in f:
            parts = line.split()
            if not parts:
                continue
            n = int(parts[0])
            ids.extend(int(v) for v in parts[1: 1 + n])
            offs.append(len(ids))
    return rows, np.array(offs, dtype=np.uint64), np.array(ids, dtype=np.uint64)
