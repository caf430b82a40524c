"""Mode-B oracle: a CPU restatement of the reference's k-mer table build from KMC databases.

TEST INFRASTRUCTURE ONLY — imported by tests/ as the checker, never by the product.

Restated from (paths under /root/reference):
  read_kmc        CKMCFile::OpenForListing / ReadParamsFrom_prefix_file_buf / ReadNextKmer
                  (kmer/kmc_api/kmc_file.cpp:66-310, :438-532): versions 0 (KMC1) and 0x200
                  (KMC2/3); records outside [min_count, max_count] are skipped
  build_khtable   buildKHtable with kmc = false (io/ioHT.cc:83-199) over KmcRead / KmcCount
                  (kmer/kmc_reader.cc:26-169): the union of canonical k-mers (Kmer twin / operator<,
                  kmer/Kmer.cc:76-187) over every sample, per-sample counts summed and clamped at
                  65535, coverage = float sum of log(count) in file order.  A database listing
                  fewer k-mers than its total adds the all-A k-mer (the default-constructed Kmer
                  left in KmcRead's vector).
The reference's row order is libcuckoo's table order; rows here are in first-appearance order
(sample order, then file order), the order the product writes.  Pinned by tests/golden/mode_b.json
(the reference's own outputs, compared as rows keyed by k-mer).
"""
from __future__ import annotations

import math
import struct

import numpy as np


def read_kmc(name: str):
    """(k, [(kmer value with s[0] most significant, count)], total_kmers) as listed."""
    with open(name + ".kmc_pre", "rb") as f:
        pre = f.read()
    with open(name + ".kmc_suf", "rb") as f:
        suf = f.read()
    assert pre[:4] == b"KMCP" and pre[-4:] == b"KMCP" and suf[:4] == b"KMCS" and suf[-4:] == b"KMCS"
    size = len(pre) - 8
    version = struct.unpack_from("<I", pre, len(pre) - 12)[0]
    header_offset = pre[len(pre) - 8]
    if version == 0x200:
        size -= 4
        h = len(pre) - (header_offset + 8)
        k, mode, counter_size, p, sig_len, min_count, max_count = struct.unpack_from("<7I", pre, h)
        total = struct.unpack_from("<Q", pre, h + 28)[0]
        sig_size = (1 << (2 * sig_len)) + 1
        lut_bytes = size - (sig_size * 4 + header_offset + 8)
        lut = list(struct.unpack_from("<%dQ" % ((lut_bytes + 8) // 8), pre, 4))
        lut[lut_bytes // 8] = total + 1
    elif version == 0:
        n = (size - 4) // 8
        buf = list(struct.unpack_from("<%dQ" % n, pre, 4))
        size -= 4
        hi = (size - header_offset) // 8
        k, mode = buf[hi] & 0xFFFFFFFF, buf[hi] >> 32
        counter_size, p = buf[hi + 1] & 0xFFFFFFFF, buf[hi + 1] >> 32
        min_count, max_count = buf[hi + 2] & 0xFFFFFFFF, buf[hi + 2] >> 32
        total = buf[hi + 3]
        max_count += buf[hi + 4] & 0xFFFFFFFF00000000
        lut = buf
        lut[hi] = total + 1
    else:
        raise ValueError("KMC version %#x" % version)
    assert mode == 0
    sufix_size = (k - p) // 4
    rec = sufix_size + counter_size
    mask = (1 << (2 * p)) - 1
    out = []
    pi = 0
    data = suf[4:-4]
    assert len(data) == total * rec, (len(data), total, rec)
    for r in range(total):
        if r == lut[pi + 1]:
            pi += 1
            while lut[pi] == lut[pi + 1]:
                pi += 1
        o = r * rec
        sv = int.from_bytes(data[o:o + sufix_size], "big") if sufix_size else 0
        cnt = int.from_bytes(data[o + sufix_size:o + rec], "little")
        if min_count <= cnt <= max_count:
            out.append((((pi & mask) << (2 * (k - p))) | sv, cnt))
    return k, out, total


def image(v: int, k: int) -> int:
    """KMC value (s[0] most significant) -> the reference Kmer's 8-byte image (base i at bits 2i)."""
    r = 0
    for i in range(k):
        r |= ((v >> (2 * (k - 1 - i))) & 3) << (2 * i)
    return r


def canonical(img: int, k: int) -> int:
    t = 0
    for i in range(k):
        t |= (3 - ((img >> (2 * (k - 1 - i))) & 3)) << (2 * i)
    return img if img.to_bytes(8, "little") < t.to_bytes(8, "little") else t


def build_khtable(names, k: int):
    """(reps in first-appearance order, counts [d][kmap] uint16, log text)."""
    order, index = [], {}
    listed = []
    for nm in names:
        kk, recs, total = read_kmc(nm)
        reps = [canonical(image(v, kk), k) for v, _ in recs]
        listed.append((reps, [c for _, c in recs]))
        for r in reps:
            if r not in index:
                index[r] = len(order)
                order.append(r)
        if len(recs) < total and 0 not in index:
            index[0] = len(order)
            order.append(0)
    kmap = len(order)
    counts = np.zeros((len(names), kmap), np.uint16)
    log = "%d" % kmap
    for j, (reps, cnts) in enumerate(listed):
        acc = np.zeros(kmap, np.uint64)
        cov = np.float32(0.0)
        for r, c in zip(reps, cnts):
            acc[index[r]] = min(int(acc[index[r]]) + c, 65535)
            cov = np.float32(np.float64(cov) + math.log(c))
        counts[j] = acc.astype(np.uint16)
        log += "\t%f" % float(cov)
    return order, counts, log


def rows_by_kmer(reps, counts) -> dict:
    """{rep: tuple of per-sample counts} (the order-free view of kmer_set.hex + kmer_count.bin)."""
    return {int(r): tuple(int(x) for x in counts[:, i]) for i, r in enumerate(reps)}


def read_outputs(dirpath: str, d: int):
    import os

    with open(os.path.join(dirpath, "kmer_count.log")) as f:
        log = f.read()
    kmap = int(log.split()[0])
    reps = np.fromfile(os.path.join(dirpath, "kmer_set.hex"), np.uint64, count=kmap)
    counts = np.fromfile(os.path.join(dirpath, "kmer_count.bin"), np.uint16).reshape(d, kmap)
    return reps, counts, log
