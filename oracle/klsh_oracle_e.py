"""Mode-E oracle: a CPU restatement of the reference's differential test + read extraction.

TEST INFRASTRUCTURE ONLY — imported by tests/ as the checker, never by the product
(kmerlsh_amd/), which runs the k-mer vote on the GPU and fails loudly without it.

Restated from (paths under /root/reference):
  read_fastq      utils/fastq.cc:28-67 (FastqFile::read_next / read) over kmer/kseq.h:60-200
                  (this kseq variant: the name is the whole header line; the sequence keeps
                  isgraph() characters up to '>', '+' or '@'; the quality is the next seq.l
                  characters in [33, 127], one extra character consumed; chars are signed)
  check_reads     IOFQ::CheckRead io/ioFastQ.cc:5-76 with Kmer (kmer/Kmer.cc:115-135 set_kmer,
                  :150-187 twin, :210-237 forwardBase, :76-78 operator< = memcmp): vectorised in
                  numpy over all k-mer positions (integer arithmetic)
  wrs_groups      AB::WRS function/funcAB.cc:73-109.  The t-test p-values come from scipy's
                  Student t distribution, not ALGLIB's bits: the decisions only, which the
                  fixtures' p-values are far from the threshold for.  (The product's ALGLIB
                  restatement is pinned bit-for-bit by tests/golden/ttest.npz, made by ALGLIB.)
  mode_e          app/kmerLSH.cc:521-580 + IOMat::ReadClusterAll io/ioMatrix.cc:48-119 +
                  IOFQ::Extracting / ReadExtract io/ioFastQ.cc:78-195
Pinned by tests/golden/mode_e.json (output md5s of the reference CLI itself).
"""
from __future__ import annotations

import gzip
import os

import numpy as np


def _open(path: str) -> bytes:
    with open(path, "rb") as f:
        head = f.read(2)
    if head == b"\x1f\x8b":
        with gzip.open(path, "rb") as f:
            return f.read()
    with open(path, "rb") as f:
        return f.read()


def read_fastq(path: str):
    """[(name, seq, qual)] as bytes, in file order (kseq_read until -1 / -2)."""
    data = _open(path)
    n = len(data)
    pos = 0
    out = []
    last = 0

    def getc():
        nonlocal pos
        if pos >= n:
            return -1
        b = data[pos]
        pos += 1
        return b - 256 if b >= 128 else b

    while True:
        if last == 0:
            c = getc()
            while c != -1 and c not in (62, 64):
                c = getc()
            if c == -1:
                break
            last = c
        if pos >= n:
            break
        nl = data.find(b"\n", pos)
        if nl < 0:
            name, pos = data[pos:], n
        else:
            name, pos = data[pos:nl], nl + 1
        seq = bytearray()
        c = getc()
        while c != -1 and c not in (62, 43, 64):
            if 33 <= c <= 126:
                seq.append(c)
            c = getc()
        if c in (62, 64):
            last = c
        if c != 43:
            out.append((bytes(name), bytes(seq), b""))
            continue
        c = getc()
        while c != -1 and c != 10:
            c = getc()
        if c == -1:
            break  # -2: truncated record ends the file
        qual = bytearray()
        c = getc()
        while c != -1 and len(qual) < len(seq):
            if 33 <= c <= 127:
                qual.append(c)
            c = getc()
        last = 0
        if len(qual) != len(seq):
            break
        out.append((bytes(name), bytes(seq), bytes(qual)))
    return out


_CODE = np.zeros(256, np.uint64)
_CODE[ord("C")], _CODE[ord("G")], _CODE[ord("T")] = 1, 2, 3


def canonical_kmers(seq: bytes, k: int) -> np.ndarray:
    """rep = (km < twin) ? km : twin for every k-mer position (uint64 images of the 8 bytes)."""
    c = _CODE[np.frombuffer(seq, np.uint8)]
    npos = len(seq) - k + 1
    if npos <= 0:
        return np.zeros(0, np.uint64)
    fwd = np.zeros(npos, np.uint64)
    rc = np.zeros(npos, np.uint64)
    for i in range(k):
        fwd |= c[i:i + npos] << np.uint64(2 * i)
        rc |= (np.uint64(3) - c[i:i + npos]) << np.uint64(2 * (k - 1 - i))
    fb = fwd.byteswap()
    rb = rc.byteswap()
    return np.where(fb < rb, fwd, rc)


def check_reads(seqs, kset: np.ndarray, k: int, vote: float):
    """(hits, flags) per read; kset: uint64 k-mer images (any order, duplicates allowed)."""
    keys = np.unique(np.asarray(kset, np.uint64))
    hits = np.zeros(len(seqs), np.uint32)
    flags = np.zeros(len(seqs), np.uint8)
    for r, s in enumerate(seqs):
        if len(s) < k + 10:
            continue
        reps = canonical_kmers(s, k)
        h = int(np.isin(reps, keys, assume_unique=False).sum())
        hits[r] = h
        flags[r] = 1 if np.float32(h) / np.float32(len(s) - k + 1) > np.float32(vote) else 0
    return hits, flags


def extract_bytes(records, flags) -> bytes:
    out = []
    for (name, seq, qual), f in zip(records, flags):
        if f:
            out.append(b"@" + name + b"\n" + seq + b"\n+\n" + qual + b"\n")
    return b"".join(out)


def read_cluster_all(file_name: str, d: int):
    """(values [line_cnt][d] f32, member-id lists) as IOMat::ReadClusterAll pairs them."""
    vals = np.fromfile(file_name, np.float32)
    line_cnt = vals.size // d
    vals = vals[: line_cnt * d].reshape(line_cnt, d)
    ids = []
    with open(file_name + ".clust") as f:
        for line in f:
            parts = line.split()
            n = int(parts[0]) if parts else 0
            got = [int(x) for x in parts[1:1 + n]]
            ids.append(got + [0] * (n - len(got)))
    return vals, ids


def wrs_groups(values: np.ndarray, id_lists, n1: int, n2: int, pval: float, size_thresh: int):
    from scipy import stats

    g = np.zeros(len(id_lists), np.uint8)
    p = np.float64(np.float32(pval))
    for c, ids in enumerate(id_lists):
        if not len(ids) > size_thresh:
            continue
        x = values[c, :n1].astype(np.float64)
        y = values[c, n1:n1 + n2].astype(np.float64)
        if n1 <= 0 or n2 <= 0:
            left = right = 1.0
        else:
            xm = x[0] if np.all(x == x[0]) else x.sum() / n1
            ym = y[0] if np.all(y == y[0]) else y.sum() / n2
            s = 0.0
            if n1 + n2 > 2:
                s = np.sqrt((((x - xm) ** 2).sum() + ((y - ym) ** 2).sum())
                            * (1.0 / n1 + 1.0 / n2) / (n1 + n2 - 2))
            if s == 0:
                left = 1.0 if xm >= ym else 0.0
                right = 1.0 if xm <= ym else 0.0
            else:
                cdf = stats.t.cdf((xm - ym) / s, n1 + n2 - 2)
                left, right = cdf, 1.0 - cdf
        if left <= p:
            g[c] = 2
        elif right <= p:
            g[c] = 1
    return g


def mode_e(dirpath: str, k: int, size_thresh: int, pval: float, vote: float,
           clust_file: str = "clustering_result.txt", out1: str = "A", out2: str = "B"):
    """The whole mode E in `dirpath`; returns {output file name: bytes} and the id-set sizes."""
    def samples(list_file):
        with open(os.path.join(dirpath, list_file)) as f:
            return [ln.split()[0] if ln.split() else "" for ln in f.read().splitlines()]

    s1, s2 = samples("a.txt"), samples("b.txt")
    n1, n2 = len(s1), len(s2)
    vals, id_lists = read_cluster_all(os.path.join(dirpath, clust_file), n1 + n2)
    g = wrs_groups(vals, id_lists, n1, n2, pval, size_thresh)
    set1, set2 = set(), set()
    for c, ids in enumerate(id_lists):
        if g[c] == 1:
            set1.update(ids)
        elif g[c] == 2:
            set2.update(ids)
    with open(os.path.join(dirpath, "kmer_count.log")) as f:
        kmap = int(f.read().split()[0])
    km = np.fromfile(os.path.join(dirpath, "kmer_set.hex"), np.uint64, count=kmap)
    k1 = np.array([km[i] for i in range(kmap) if i in set1], np.uint64)
    k2 = np.array([km[i] for i in range(kmap) if i not in set1 and i in set2], np.uint64)
    outs = {}
    for prefix, names, ks in ((out1, s1, k1), (out2, s2, k2)):
        for nm in names:
            recs = read_fastq(os.path.join(dirpath, nm))
            _, flags = check_reads([r[1] for r in recs], ks, k, vote)
            outs["%s_%s" % (prefix, os.path.basename(nm))] = extract_bytes(recs, flags)
    return outs, (len(set1), len(set2))
