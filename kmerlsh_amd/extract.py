"""Host-side mirror of the reference's mode-E interface, driving the gfx950 engine.

Reference interface mirrored (same names and argument meaning):
  void AB::WRS(unordered_set<uint64_t>* group1, unordered_set<uint64_t>* group2,
               Abundance* abundance, int num_sample1, int num_sample2, float pvalue_thresh,
               int size_thresh)                                       function/funcAB.cc:73-109
  void IOMat::ReadClusterAll(vector<Abundance*>*, int num_samples, string file_name, bool)
                                                                       io/ioMatrix.cc:48-119
  void IOFQ::CheckRead(uset_t*, vector<ReadEntry>&, vector<int>& record_vec, ...,
                       float kmer_vote)                                io/ioFastQ.cc:5-76
  void IOFQ::ReadExtract(uset_t*, vector<string>& files, string output, float kmer_vote, ...)
                                                                       io/ioFastQ.cc:78-159
  void IOFQ::Extracting(vector<string> samples, uset_t*, string out, int num_threads,
                        float kmer_vote, bool verbose)                 io/ioFastQ.cc:161-195

The t-test runs on the host (klsh_wrs: ALGLIB restated, bit-exact); the k-mer vote over the reads
runs on the GPU (klsh_check_reads / klsh_extract_fastq).  No CPU fallback: without the library or a
gfx950 device every GPU entry point raises.  k-mers are the reference's 8-byte Kmer images as
little-endian uint64 (kmer_set.hex layout, kmer/Kmer.cc:307).
"""
from __future__ import annotations

import os

import numpy as np

from . import _native
from .cluster import Abundance


def ReadClusterAll(num_samples: int, file_name: str = "clustering_result.txt"):
    """Abundances from <file_name> (fp32 rows) and <file_name>.clust (member lists), paired line
    by line; a line with fewer ids than its count keeps zeros (the reference's vector(n))."""
    vals = np.fromfile(file_name, np.float32)
    line_cnt = vals.size // num_samples if num_samples else 0
    vals = vals[: line_cnt * num_samples].reshape(line_cnt, num_samples)
    out = []
    with open(file_name + ".clust") as f:
        for loc, line in enumerate(f):
            parts = line.split()
            n = int(parts[0]) if parts else 0
            ids = [int(x) for x in parts[1:1 + n]]
            out.append(Abundance(vals[loc], ids + [0] * (n - len(ids))))
    return out


def WRS(group1: set, group2: set, abundance: Abundance, num_sample1: int, num_sample2: int,
        pvalue_thresh: float, size_thresh: int) -> None:
    """One cluster's test; its ids join group2 (lefttail <= p) or group1 (righttail <= p)."""
    g = _native.wrs(np.asarray(abundance._values, np.float32)[None, :],
                    np.array([len(abundance._ids)], np.uint64), num_sample1, num_sample2,
                    pvalue_thresh, size_thresh)[0]
    if g == 2:
        group2.update(abundance._ids)
    elif g == 1:
        group1.update(abundance._ids)


def wrs_all(abundances, num_sample1: int, num_sample2: int, pvalue_thresh: float,
            size_thresh: int):
    """WRS over every cluster in one call: (group1 ids, group2 ids)."""
    d = num_sample1 + num_sample2
    vals = np.array([a._values for a in abundances], np.float32).reshape(len(abundances), d)
    g = _native.wrs(vals, np.array([len(a._ids) for a in abundances], np.uint64), num_sample1,
                    num_sample2, pvalue_thresh, size_thresh)
    g1, g2 = set(), set()
    for a, gg in zip(abundances, g):
        if gg == 1:
            g1.update(a._ids)
        elif gg == 2:
            g2.update(a._ids)
    return g1, g2


def read_kmer_set(kmap_size: int, path: str = "kmer_set.hex") -> np.ndarray:
    """The k-mer of every row of kmer_count.bin, in row order (8 bytes each)."""
    return np.fromfile(path, np.uint64, count=kmap_size)


def CheckRead(kset: "_native.KmerSet", reads, k: int, kmer_vote: float) -> np.ndarray:
    """record_vec for a list of read sequences (bytes): 1 where the k-mer vote passes."""
    return kset.check_reads(list(reads), k, kmer_vote)[1].astype(np.int32)


def ReadExtract(kset: "_native.KmerSet", files, output: str, k: int, kmer_vote: float) -> dict:
    """The passing records of the file(s) written to `output` (the reference reads one file)."""
    stats = None
    for path in files:
        stats = kset.extract_fastq(path, output, k, kmer_vote)
    return stats or {}


def Extracting(samples, kset: "_native.KmerSet", out: str, k: int, kmer_vote: float,
               verbose: bool = False) -> list:
    """ReadExtract per sample into <out>_<basename(sample)>; returns the per-file stats."""
    stats = []
    for path in samples:
        filename = out + "_" + os.path.basename(path)
        if verbose:
            print("writing to " + filename)
        stats.append(kset.extract_fastq(path, filename, k, kmer_vote))
    return stats
