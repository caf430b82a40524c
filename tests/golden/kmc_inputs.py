"""KMC k-mer databases for mode-B fixtures (TEST INFRASTRUCTURE ONLY).

Writes .kmc_pre / .kmc_suf pairs in the two layouts the reference's vendored KMC API lists
(kmer/kmc_api/kmc_file.cpp:66-310, :438-532): KMC1 (version 0: prefix LUT + 5-word header) and
KMC2/3 (version 0x200: per-signature-bin LUTs + signature map + packed header).  A record is the
k-mer's suffix after the lut_prefix_length-symbol prefix, big-endian 2-bit symbols, then a
little-endian counter of counter_size bytes.  `write_case(dir, case)` also writes a.txt/b.txt
("<fastq> <kmc db name>" lines) for the reference CLI's mode B (`-M B --only`).
The databases are drawn from a splitmix64 stream: byte-reproducible anywhere.
"""
from __future__ import annotations

import os
import struct

from mode_e_inputs import SplitMix, revcomp

CASES = {
    # k = 21, KMC1 layout, 3 + 3 samples, 2-byte counters
    "b21": dict(k=21, version=0, p=9, counter_size=2, n1=3, n2=3, genomes=5, glen=1500, seed=31,
                canonical=True, min_count=1, bins=1, big_counts=False),
    # k = 31, KMC2 layout with 3 signature bins, 1-byte counters, min_count 3 (filtered records)
    "b31": dict(k=31, version=0x200, p=11, counter_size=1, n1=2, n2=2, genomes=4, glen=1200,
                seed=37, canonical=True, min_count=3, bins=3, big_counts=False),
    # k = 32, KMC1, 4-byte counters near 65535 (saturation), k-mers listed on both strands
    "b32": dict(k=32, version=0, p=12, counter_size=4, n1=2, n2=3, genomes=4, glen=1000, seed=41,
                canonical=False, min_count=1, bins=1, big_counts=True),
}

CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def kmer_value(s: str) -> int:
    """KMC's k-mer as an integer: s[0] the most significant symbol (kmer_api.h:380-395)."""
    v = 0
    for ch in s:
        v = (v << 2) | CODE[ch]
    return v


def write_db(path: str, k: int, records, version: int, p: int, counter_size: int,
             min_count: int, max_count: int, bins: int = 1, sig_len: int = 5) -> None:
    """records: [(kmer string, count)] (any order; duplicates allowed).  Bin of a record: a hash of
    the k-mer (version 0x200 only); within a bin, records sorted by (prefix, suffix)."""
    suf_sym = k - p
    assert suf_sym % 4 == 0 and suf_sym >= 0
    sufix_size = suf_sym // 4
    nb = bins if version == 0x200 else 1
    per_bin = [[] for _ in range(nb)]
    for s, c in records:
        v = kmer_value(s)
        b = (v * 0x9E3779B97F4A7C15 >> 61) % nb if nb > 1 else 0
        per_bin[b].append((v >> (2 * suf_sym), v & ((1 << (2 * suf_sym)) - 1), c))
    import numpy as np

    L = 1 << (2 * p)
    luts = []
    recs = bytearray()
    total = 0
    for b in range(nb):
        rs = sorted(per_bin[b])
        counts_per_prefix = np.bincount(np.array([pre for pre, _, _ in rs], np.int64),
                                        minlength=L).astype(np.uint64)
        # lut[i] = total + records with a smaller prefix (an exclusive running sum)
        luts.append(np.uint64(total) + np.concatenate([[0], np.cumsum(counts_per_prefix)[:-1]]).astype(np.uint64))
        for pre, suf, c in rs:
            recs += suf.to_bytes(sufix_size, "big") if sufix_size else b""
            recs += int(c).to_bytes(counter_size, "little")
        total += len(rs)
    lut = np.concatenate(luts).astype("<u8")
    with open(path + ".kmc_suf", "wb") as f:
        f.write(b"KMCS" + bytes(recs) + b"KMCS")
    both = 0  # stored flag 0 = "both strands" (the reader negates it)
    with open(path + ".kmc_pre", "wb") as f:
        f.write(b"KMCP")
        f.write(lut.tobytes())
        if version == 0:
            hdr = struct.pack("<5Q", k | (0 << 32), counter_size | (p << 32),
                              min_count | ((max_count & 0xFFFFFFFF) << 32), total, both)
            f.write(hdr)
            f.write(struct.pack("<I", len(hdr)))
        else:
            f.write(struct.pack("<Q", 0))  # overwritten by the reader with total + 1
            f.write(struct.pack("<%dI" % ((1 << (2 * sig_len)) + 1), *([0] * ((1 << (2 * sig_len)) + 1))))
            hdr = struct.pack("<7IQB", k, 0, counter_size, p, sig_len, min_count, max_count, total, both)
            hdr += b"\0" * 3 + struct.pack("<I", 0x200)  # pad, then the version word at END-12
            f.write(hdr)
            f.write(struct.pack("<I", len(hdr)))
        f.write(b"KMCP")


def write_case(dirpath: str, case: str) -> dict:
    c = CASES[case]
    k = c["k"]
    rng = SplitMix(c["seed"])
    genomes = ["".join("ACGT"[rng.below(4)] for _ in range(c["glen"])) for _ in range(c["genomes"])]
    d = c["n1"] + c["n2"]
    names = []
    for j in range(d):
        seen = {}
        for g, s in enumerate(genomes):
            if rng.below(3) == 0:  # this sample lacks genome g
                continue
            for pos in range(len(s) - k + 1):
                if rng.below(4) == 0:
                    continue
                km = s[pos:pos + k]
                if c["canonical"]:
                    km = min(km, revcomp(km))  # KMC's canonical form (lexicographic)
                elif rng.below(2):
                    km = revcomp(km)
                cnt = (60000 + rng.below(20000)) if c["big_counts"] and rng.below(3) == 0 else 1 + rng.below(200 if c["counter_size"] > 1 else 250)
                seen[km] = seen.get(km, 0) + cnt
        recs = list(seen.items())
        if c["counter_size"] == 1:
            recs = [(km, min(cnt, 255)) for km, cnt in recs]
        recs += [("".join("ACGT"[rng.below(4)] for _ in range(k)), 1 + rng.below(5)) for _ in range(50)]
        name = "db%d" % j
        write_db(os.path.join(dirpath, name), k, recs, c["version"], c["p"], c["counter_size"],
                 c["min_count"], 0xFFFFFFFF if c["counter_size"] == 4 else (1 << (8 * c["counter_size"])) - 1,
                 bins=c["bins"])
        names.append(name)
    with open(os.path.join(dirpath, "a.txt"), "w") as f:
        f.write("".join("s%d.fq %s\n" % (j, names[j]) for j in range(c["n1"])))
    with open(os.path.join(dirpath, "b.txt"), "w") as f:
        f.write("".join("s%d.fq %s\n" % (j, names[j]) for j in range(c["n1"], d)))
    return dict(c, d=d, names=names)


def cli_args(case: str) -> list:
    return ["-a", "a.txt", "-b", "b.txt", "-o", "A", "-p", "B", "-K", str(CASES[case]["k"]), "-M", "B",
            "--only", "--verbose", "-T", "1"]


# Large mode-B cases (the reference's libcuckoo table under load): KMC1 databases of random
# k-mers drawn from a vectorised splitmix64 stream, written with numpy (the per-record writer above
# is too slow for 10^5..10^6 records).  "bl_fill": ~470K distinct k-mers, one table of 2^16 8-slot
# buckets at ~90 % load (long cuckoo paths); "bl_grow": ~640K, past what that table holds, so it
# doubles once.
BIG_CASES = {
    "bl_fill": dict(k=31, p=11, samples=2, per_sample=276_000, overlap=0.43, seed=101),
    "bl_grow": dict(k=31, p=11, samples=2, per_sample=400_000, overlap=0.40, seed=103),
}


def _splitmix_np(seed: int, n: int):
    import numpy as np

    x = (np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) + np.uint64(seed)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def write_big_case(dirpath: str, case: str) -> dict:
    """Sample j lists per_sample k-mers: an `overlap` share drawn from a pool common to all
    samples, the rest its own; counts 1..200 (1-byte counters), KMC1 layout, sorted records."""
    import numpy as np

    c = BIG_CASES[case]
    k, p, n = c["k"], c["p"], c["per_sample"]
    kmask = np.uint64((1 << (2 * k)) - 1)
    shared = _splitmix_np(c["seed"], n) & kmask
    names = []
    for j in range(c["samples"]):
        own = _splitmix_np(c["seed"] * 7919 + j + 1, n) & kmask
        pick = _splitmix_np(c["seed"] * 104729 + j, n) % np.uint64(1000) < np.uint64(int(c["overlap"] * 1000))
        vals = np.unique(np.where(pick, shared, own))
        cnt = (_splitmix_np(c["seed"] + 17 * j, vals.size) % np.uint64(200) + np.uint64(1)).astype(np.uint8)
        suf_sym = k - p
        pre = (vals >> np.uint64(2 * suf_sym)).astype(np.int64)
        suf = vals & np.uint64((1 << (2 * suf_sym)) - 1)
        sb = suf_sym // 4
        rec = np.zeros((vals.size, sb + 1), np.uint8)
        for b in range(sb):  # big-endian suffix bytes
            rec[:, b] = ((suf >> np.uint64(8 * (sb - 1 - b))) & np.uint64(0xFF)).astype(np.uint8)
        rec[:, sb] = cnt
        lut = np.zeros(1 << (2 * p), np.uint64)
        np.add.at(lut, pre, 1)
        lut = np.concatenate([[0], np.cumsum(lut)[:-1]]).astype("<u8")
        name = "db%d" % j
        path = os.path.join(dirpath, name)
        with open(path + ".kmc_suf", "wb") as f:
            f.write(b"KMCS" + rec.tobytes() + b"KMCS")
        with open(path + ".kmc_pre", "wb") as f:
            f.write(b"KMCP")
            f.write(lut.tobytes())
            hdr = struct.pack("<5Q", k, 1 | (p << 32), 1 | (255 << 32), vals.size, 0)
            f.write(hdr)
            f.write(struct.pack("<I", len(hdr)))
            f.write(b"KMCP")
        names.append(name)
    with open(os.path.join(dirpath, "a.txt"), "w") as f:
        f.write("s0.fq %s\n" % names[0])
    with open(os.path.join(dirpath, "b.txt"), "w") as f:
        f.write("".join("s%d.fq %s\n" % (j, names[j]) for j in range(1, c["samples"])))
    return dict(c, d=c["samples"], names=names)


def big_cli_args(case: str) -> list:
    return ["-a", "a.txt", "-b", "b.txt", "-o", "A", "-p", "B", "-K", str(BIG_CASES[case]["k"]),
            "-M", "B", "--only", "--verbose", "-T", "1"]
