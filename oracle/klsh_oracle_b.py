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
  cuckoo_order    the row order: the reference's libcuckoo table (hash/HashTables.h:22, the
                  vendored utils/libcuckoo/cuckoohash_map.hh: 8-slot buckets, 2^16 of them to start,
                  index_hash / alt_index :893-908, cuckoo_insert :1428-1483, BFS slot_search
                  :983-1022, cuckoopath_move :1124-1176, cuckoo_expand_simple :1627-1667) after
                  KmcRead's inserts at -T 1 (kmer/kmc_reader.cc:5-20, 66-70) — a duplicate insert
                  changes nothing, so it is the distinct k-mers inserted in first-appearance order —
                  iterated bucket by bucket, slot by slot (io/ioHT.cc:140-149).  Kmer::hash()
                  (kmer/Kmer.cc:138-147) is hash/hash.cc's early MurmurHash3_x64_128 revision.
Pinned by tests/golden/mode_b.json: the reference CLI's own kmer_set.hex / kmer_count.bin md5s
(byte for byte) on the small cases and on a table loaded to 95.6 % (long cuckoo paths).
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
        lut = np.frombuffer(pre, "<u8", (lut_bytes + 8) // 8, 4).astype(np.uint64)
        lut[lut_bytes // 8] = total + 1
        lut = lut[:lut_bytes // 8 + 1]
    elif version == 0:
        n = (size - 4) // 8
        buf = np.frombuffer(pre, "<u8", n, 4).astype(np.uint64)
        size -= 4
        hi = (size - header_offset) // 8
        w = [int(x) for x in buf[hi:hi + 5]]
        k, mode = w[0] & 0xFFFFFFFF, w[0] >> 32
        counter_size, p = w[1] & 0xFFFFFFFF, w[1] >> 32
        min_count, max_count = w[2] & 0xFFFFFFFF, w[2] >> 32
        total = w[3]
        max_count += w[4] & 0xFFFFFFFF00000000
        lut = buf[:hi + 1].copy()
        lut[hi] = total + 1
    else:
        raise ValueError("KMC version %#x" % version)
    assert mode == 0
    sufix_size = (k - p) // 4
    rec = sufix_size + counter_size
    mask = (1 << (2 * p)) - 1
    data = suf[4:-4]
    assert len(data) == total * rec, (len(data), total, rec)
    # record r's prefix: the reader's LUT walk (skipping empty prefixes) = the last LUT entry <= r
    pis = np.searchsorted(lut, np.arange(total, dtype=np.uint64), side="right") - 1
    recs = np.frombuffer(data, np.uint8).reshape(total, rec) if total else np.zeros((0, rec), np.uint8)
    sv = np.zeros(total, np.uint64)
    for b in range(sufix_size):  # big-endian suffix
        sv = (sv << np.uint64(8)) | recs[:, b].astype(np.uint64)
    cnt = np.zeros(total, np.uint64)
    for b in range(counter_size):  # little-endian counter
        cnt |= recs[:, sufix_size + b].astype(np.uint64) << np.uint64(8 * b)
    vals = ((pis.astype(np.uint64) & np.uint64(mask)) << np.uint64(2 * (k - p))) | sv
    keep = (cnt >= np.uint64(min_count)) & (cnt <= np.uint64(max_count))
    out = list(zip(vals[keep].tolist(), cnt[keep].tolist()))
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


M64 = (1 << 64) - 1


def kmer_hash(img: int, k: int) -> int:
    """Kmer::hash(): the first word of hash/hash.cc's MurmurHash3_x64_128 (seed 0) over the
    Kmer's (k+3)/4 bytes — one tail block (k1 = those bytes little-endian, k2 = 0)."""
    nb = (k + 3) // 4

    def rotl(v, r):
        return ((v << r) | (v >> (64 - r))) & M64

    def fmix(x):
        x ^= x >> 33
        x = (x * 0xff51afd7ed558ccd) & M64
        x ^= x >> 33
        x = (x * 0xc4ceb9fe1a85ec53) & M64
        return x ^ (x >> 33)

    h1, h2 = 0x9368e53c2f6af274, 0x586dcd208f7cd3fd
    c1, c2 = 0x87c37b91114253d5, 0x4cf5ad432745937f
    k1 = img & ((1 << (8 * nb)) - 1)
    k1 = (rotl((k1 * c1) & M64, 23) * c2) & M64       # bmix64 (hash.cc:73-92), k2 = 0
    h1 = ((h1 ^ k1) + h2) & M64
    h2 = (rotl(h2, 41) + h1) & M64
    h1 = (h1 * 3 + 0x52dce729) & M64
    h2 = (h2 * 3 + 0x38495ab5) & M64
    h2 ^= nb                                            # finalization (hash.cc:160-172)
    h1 = (h1 + h2) & M64
    h2 = (h2 + h1) & M64
    return (fmix(h1) + fmix(h2)) & M64


def cuckoo_order(reps, k: int, hashpower: int = 16):
    """Indices of `reps` (distinct, in insertion order) in the table's iteration order, and the
    final hash power."""
    SLOTS, MAXD, QN = 8, 4, 501
    hv = [kmer_hash(int(r), k) for r in reps]
    st = {"hp": hashpower}
    tab = [-1] * (SLOTS << hashpower)

    def alt(h, b):
        m = (1 << st["hp"]) - 1
        return (b ^ ((((h >> st["hp"]) + 1) * 0x5bd1e995) & M64)) & m

    def free_slot(b):
        for s in range(SLOTS):
            if tab[b * SLOTS + s] < 0:
                return s
        return -1

    def search(a, b):  # slot_search: (bucket, pathcode, depth) or None
        q = [None] * QN
        first, last = 0, 0
        nxt = lambda i: 0 if i == QN - 1 else i + 1  # noqa: E731
        q[last] = (a, 0, 0); last = nxt(last)          # noqa: E702
        q[last] = (b, 1, 0); last = nxt(last)          # noqa: E702
        while nxt(last) != first:
            xb, xp, xd = q[first]
            first = nxt(first)
            s = 0
            while s < SLOTS and nxt(last) != first:
                e = tab[xb * SLOTS + s]
                if e < 0:
                    return xb, xp * SLOTS + s, xd
                yb = alt(hv[e], xb)
                yp, yd = xp * SLOTS + s, xd + 1
                j = free_slot(yb)
                if j >= 0:
                    return yb, yp * SLOTS + j, yd
                if yd != MAXD:
                    q[last] = (yb, yp, yd)
                    last = nxt(last)
                s += 1
        return None

    def insert(e):
        while True:
            m = (1 << st["hp"]) - 1
            a = hv[e] & m
            b = alt(hv[e], a)
            for bk in (a, b):
                s = free_slot(bk)
                if s >= 0:
                    tab[bk * SLOTS + s] = e
                    return
            found = search(a, b)
            if found is None:
                expand()
                continue
            _, code, depth = found
            slots = [0] * (depth + 1)
            for i in range(depth, -1, -1):
                slots[i] = code % SLOTS
                code //= SLOTS
            buckets = [a if code == 0 else b]
            for i in range(1, depth + 1):
                pe = tab[buckets[i - 1] * SLOTS + slots[i - 1]]
                buckets.append(alt(hv[pe], buckets[i - 1]))
            for dd in range(depth, 0, -1):
                tab[buckets[dd] * SLOTS + slots[dd]] = tab[buckets[dd - 1] * SLOTS + slots[dd - 1]]
                tab[buckets[dd - 1] * SLOTS + slots[dd - 1]] = -1
            tab[buckets[0] * SLOTS + slots[0]] = e
            return

    def expand():
        old = [v for v in tab if v >= 0]
        st["hp"] += 1
        tab[:] = [-1] * (SLOTS << st["hp"])
        for v in old:
            insert(v)

    for e in range(len(reps)):
        insert(e)
    return [v for v in tab if v >= 0], st["hp"]


def build_khtable(names, k: int, order: str = "reference"):
    """(reps, counts [d][kmap] uint16, log text); rows in the reference's libcuckoo order, or in
    first-appearance order (order="first")."""
    order_kind = order
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
    if order_kind == "reference":
        idx, _ = cuckoo_order(order, k)
        order = [order[i] for i in idx]
        counts = counts[:, idx]
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
