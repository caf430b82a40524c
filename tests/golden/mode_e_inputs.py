"""Formula-defined inputs for mode E (differential k-mers + read extraction) fixtures.

TEST INFRASTRUCTURE ONLY.  `write_case(dirpath, case)` writes, in `dirpath`, everything the
reference's mode E reads (app/kmerLSH.cc:521-580):

  a.txt / b.txt            sample lists ("<fastq path> <kmc name>" per line, io/ioHT.cc:3-19)
  <samples>.fq[.gz]        reads (FASTQ; one gzip file; CRLF, multi-line, lowercase, N, too-short
                           and empty-sequence records as edge cases)
  kmer_count.log           "<kmap_size>\\t..." (only the first number is read in mode E)
  kmer_set.hex             kmap_size k-mers, 8 raw bytes each (Kmer::writeBytes, kmer/Kmer.cc:307)
  clustering_result.txt    fp32 centroids, d per row (IOMat::ReadClusterAll, io/ioMatrix.cc:48-119)
  clustering_result.txt.clust  "<n>\\t<id>..." per cluster

Everything is drawn from a splitmix64 stream, so the files are byte-reproducible anywhere
(tests regenerate them instead of storing them).
"""
from __future__ import annotations

import gzip
import os
import struct

CASES = {
    # k = 21, 4 + 4 samples, tested clusters > 40 members, p <= 0.01, vote > 0.5
    "e21": dict(k=21, n1=4, n2=4, genomes=8, glen=2500, reads=700, seed=7, size_thresh=40,
                pval=0.01, vote=0.5, gz=(2,), crlf=(5,), multiline=(1,)),
    # k = 31, 3 + 2 samples (odd degrees of freedom), looser vote
    "e31": dict(k=31, n1=3, n2=2, genomes=6, glen=2000, reads=500, seed=11, size_thresh=30,
                pval=0.05, vote=0.3, gz=(0,), crlf=(), multiline=(3,)),
    # k = 32 (the full 64-bit word: the all-T k-mer's reverse complement is 0), 5 + 5 samples
    "e32": dict(k=32, n1=5, n2=5, genomes=6, glen=2000, reads=400, seed=23, size_thresh=30,
                pval=0.01, vote=0.4, gz=(), crlf=(7,), multiline=()),
}


class SplitMix:
    def __init__(self, seed: int):
        self.s = seed & 0xFFFFFFFFFFFFFFFF

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        return z ^ (z >> 31)

    def below(self, n: int) -> int:
        return self.next() % n

    def unif(self) -> float:
        return (self.next() >> 11) * (1.0 / (1 << 53))


CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def fwd_value(s: str, k: int) -> int:
    """Kmer::set_kmer (kmer/Kmer.cc:115-135): base i at bits 2i; anything but C/G/T is A (0)."""
    v = 0
    for i in range(k):
        v |= CODE.get(s[i], 0) << (2 * i)
    return v


def twin(v: int, k: int) -> int:
    """Kmer::twin (kmer/Kmer.cc:150-187): reverse complement."""
    r = 0
    for i in range(k):
        r |= (3 - ((v >> (2 * (k - 1 - i))) & 3)) << (2 * i)
    return r


def rep(v: int, k: int) -> int:
    """(km < tw) ? km : tw with operator< = memcmp of the 8 bytes (kmer/Kmer.cc:76-78)."""
    t = twin(v, k)
    return v if v.to_bytes(8, "little") < t.to_bytes(8, "little") else t


def revcomp(s: str) -> str:
    c = {"A": "T", "C": "G", "G": "C", "T": "A"}
    return "".join(c[x] for x in reversed(s))


def write_case(dirpath: str, case: str) -> dict:
    c = CASES[case]
    k, n1, n2 = c["k"], c["n1"], c["n2"]
    d = n1 + n2
    rng = SplitMix(c["seed"])
    genomes = ["".join("ACGT"[rng.below(4)] for _ in range(c["glen"])) for _ in range(c["genomes"])]

    # kmap: canonical k-mers of the genomes (de-duplicated) + 300 random ones
    kmers, index = [], {}
    for g, s in enumerate(genomes):
        for p in range(0, len(s) - k + 1):
            r = rep(fwd_value(s[p:p + k], k), k)
            if r not in index:
                index[r] = len(kmers)
                kmers.append((r, g))
    for _ in range(300):
        r = rep(fwd_value("".join("ACGT"[rng.below(4)] for _ in range(k)), k), k)
        if r not in index:
            index[r] = len(kmers)
            kmers.append((r, -1))
    if k == 32:  # the all-T word (never a canonical rep, never matched) and the all-A rep
        for r in (0xFFFFFFFFFFFFFFFF, 0):
            if r not in index:
                index[r] = len(kmers)
                kmers.append((r, -1))
    kmap = len(kmers)
    with open(os.path.join(dirpath, "kmer_set.hex"), "wb") as f:
        for r, _ in kmers:
            f.write(r.to_bytes(8, "little"))
    with open(os.path.join(dirpath, "kmer_count.log"), "w") as f:
        f.write("%d" % kmap + "".join("\t%f" % (1000.0 + j) for j in range(d)))

    # clusters: each genome's k-mers in chunks of 20..80 ids (interleaved order), the random
    # k-mers in one cluster; genome g's clusters lean to group A (g % 4 == 0), B (== 1), none
    by_g = {}
    for i, (_, g) in enumerate(kmers):
        by_g.setdefault(g, []).append(i)
    clusters = []
    for g in sorted(by_g):
        ids = by_g[g]
        a = 0
        while a < len(ids):
            b = min(len(ids), a + 20 + rng.below(61))
            clusters.append((g, ids[a:b]))
            a = b
    rows = []
    for ci, (g, ids) in enumerate(clusters):
        kind = (g % 4) if g >= 0 else 3
        shift = [1.5, -1.5, 0.0, 0.0][kind] * (0.2 + rng.unif())
        if ci % 11 == 5:  # constant row: s == 0 branch of studentttest2
            row = [0.25] * d
        elif ci % 13 == 7:  # group constant, means differ (s > 0 only through the other group)
            row = [0.5] * n1 + [0.5 + 0.1 * (j + 1) for j in range(n2)]
        else:
            row = [(shift if j < n1 else 0.0) + (rng.unif() - 0.5) * 2.0 for j in range(d)]
        rows.append(struct.pack("<%df" % d, *row))
    with open(os.path.join(dirpath, "clustering_result.txt"), "wb") as f:
        f.write(b"".join(rows))
    with open(os.path.join(dirpath, "clustering_result.txt.clust"), "w") as f:
        for _, ids in clusters:
            f.write("%d" % len(ids) + "".join("\t%d" % i for i in ids) + "\n")

    # reads
    names1, names2 = [], []
    for j in range(d):
        base = "s%d.fq" % j + (".gz" if j in c["gz"] else "")
        (names1 if j < n1 else names2).append(base)
        recs = []
        for r in range(c["reads"]):
            g = rng.below(len(genomes))
            ln = 40 + rng.below(121)
            p = rng.below(len(genomes[g]) - ln)
            s = genomes[g][p:p + ln]
            if rng.below(2):
                s = revcomp(s)
            s = list(s)
            for q in range(len(s)):
                u = rng.below(1000)
                if u < 8:
                    s[q] = "ACGT"[rng.below(4)]
                elif u < 10:
                    s[q] = "N"
                elif u < 12:
                    s[q] = s[q].lower()
            s = "".join(s)
            if r % 97 == 13:
                s = s[: k + 5]  # shorter than k + 10: never extracted (ioFastQ.cc:25)
            if r % 89 == 44:
                s = s[: k + 10]  # exactly k + 10: tested
            name = "r%d_%d sample=%d len=%d" % (j, r, j, len(s))
            qual = "".join(chr(33 + rng.below(41)) for _ in range(len(s)))
            if j in c["multiline"] and r % 5 == 0 and len(s) > 30:
                recs.append("@%s\n%s\n%s\n+\n%s\n%s\n" % (name, s[:30], s[30:], qual[:25], qual[25:]))
            else:
                recs.append("@%s\n%s\n+%s\n%s\n" % (name, s, "" if r % 3 else name, qual))
            if r == 50 and j == 0:
                recs.append("@empty_read\n\n+\n\n")  # seq '\0': "abnormal read entry skipped"
        text = "".join(recs)
        if j in c["crlf"]:
            text = text.replace("\n", "\r\n")
        path = os.path.join(dirpath, base)
        if base.endswith(".gz"):
            with gzip.GzipFile(path, "wb", mtime=0) as f:
                f.write(text.encode())
        else:
            with open(path, "w", newline="") as f:
                f.write(text)
    with open(os.path.join(dirpath, "a.txt"), "w") as f:
        f.write("".join("%s k%d\n" % (nm, i) for i, nm in enumerate(names1)))
    with open(os.path.join(dirpath, "b.txt"), "w") as f:
        f.write("".join("%s k%d\n" % (nm, n1 + i) for i, nm in enumerate(names2)))
    return dict(c, d=d, kmap=kmap, clusters=len(clusters), samples1=names1, samples2=names2)


def cli_args(case: str) -> list:
    """The mode-E command line (app/kmerLSH.cc:147-276 flags), outputs A_<sample> / B_<sample>."""
    c = CASES[case]
    return ["-a", "a.txt", "-b", "b.txt", "-o", "A", "-p", "B", "-K", str(c["k"]), "-M", "E", "--only",
            "--verbose", "-S", str(c["size_thresh"]), "-P", repr(c["pval"]), "-V", repr(c["vote"]),
            "-F", "clustering_result.txt", "-T", "1"]
