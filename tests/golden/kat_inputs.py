"""Formula-defined mode-C KAT inputs (SURVEY.md §8(c), table "Formula-defined KAT inputs").

No RNG is involved, so any language regenerates these byte-for-byte; the input md5s below are
the ones the survey recorded, and the output md5s are those of the seeded reference
(`oracle/_ref/kmerLSH_seeded`, KLSH_SEED=12345, -I 10 -T 1, OMP_THREAD_LIMIT=1).

Files written into a directory: kmer_count.bin (sample-major uint16 LE), kmer_count.log,
a.txt, b.txt.
"""
from __future__ import annotations

import math
import os

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def fmix32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x85EBCA6B)) & M32
    x ^= x >> np.uint64(13)
    x = (x * np.uint64(0xC2B2AE35)) & M32
    x ^= x >> np.uint64(16)
    return x


def counts_fg(n: int, s: int, g: int, shift: int) -> np.ndarray:
    """katF / katG count matrix, shape (S, N) sample-major."""
    i = np.arange(n, dtype=np.uint64)[None, :]
    j = np.arange(s, dtype=np.uint64)[:, None]
    gg = i % np.uint64(g)
    prof = np.uint64(1) + (fmix32(gg * np.uint64(s) + j + np.uint64(0x9E3779B9)) >> np.uint64(25))
    r = fmix32(i * np.uint64(s) + j + np.uint64(0x85EBCA6B)) >> np.uint64(24)
    cnt = prof + ((prof * r) >> np.uint64(shift))
    return np.minimum(cnt, 65535).astype(np.uint16)


def counts_n(n: int = 200000) -> np.ndarray:
    """katN (identical-row data that triggers nestedCluster), shape (8, N)."""
    A = np.array([400, 20, 300, 10, 500, 5, 250, 30], dtype=np.uint64)
    B = np.array([10, 300, 20, 400, 5, 500, 30, 250], dtype=np.uint64)
    i = np.arange(n, dtype=np.uint64)[None, :]
    s = np.arange(8, dtype=np.uint64)[:, None]
    v = np.where(i % np.uint64(3) == 0, B[:, None], A[:, None])
    extra = (((i * np.uint64(2654435761)) + s * np.uint64(97)) & M32) >> np.uint64(30)
    v = v + np.where(i % np.uint64(7) == 0, extra, np.uint64(0))
    return v.astype(np.uint16)


def coverage(cnt: np.ndarray) -> list[float]:
    out = []
    for row in cnt:
        acc = 0.0
        for c in row[row > 0].tolist():  # ascending i, summed in double
            acc += math.log(c)
        out.append(acc)
    return out


def write_kat(name: str, out_dir: str) -> None:
    os.makedirs(out_dir, exist_ok=True)
    if name == "katF":
        cnt = counts_fg(20000, 8, 400, 9)
        log = "%d" % cnt.shape[1] + "".join("\t%f" % c for c in coverage(cnt))
    elif name == "katG":
        cnt = counts_fg(20000, 16, 1000, 8)
        log = "%d" % cnt.shape[1] + "".join("\t%f" % c for c in coverage(cnt))
    elif name == "katN":
        cnt = counts_n()
        log = "%d" % cnt.shape[1] + "\t40000.250000" * cnt.shape[0]
    else:
        raise ValueError(name)
    S = cnt.shape[0]
    cnt.astype("<u2").tofile(os.path.join(out_dir, "kmer_count.bin"))
    with open(os.path.join(out_dir, "kmer_count.log"), "w") as f:
        f.write(log)  # no trailing newline (matches the survey md5s)
    with open(os.path.join(out_dir, "a.txt"), "w") as f:
        f.write("".join("s%d k%d\n" % (j, j) for j in range(S // 2)))
    with open(os.path.join(out_dir, "b.txt"), "w") as f:
        f.write("".join("s%d k%d\n" % (j, j) for j in range(S // 2, S)))
    os.makedirs(os.path.join(out_dir, "tmp"), exist_ok=True)


# Survey-recorded md5s; the output md5s are re-verified against the reference
# build by tests/golden/make_golden.sh and stored in tests/golden/kat_md5.json.
INPUT_MD5 = {
    "katF": ("0b784fb9b99ac84a4487a039d402190c", "12a3ac7ddc58d8f32919336dbab6793d"),
    "katG": ("48dfa143b737e6df4ac4cf49890d7572", "e2fa483c4799a43d7e9cef79021636e6"),
    "katN": ("e07415964869688e7350d2a85743e365", "d9e40a5bc8ace5cc7795cc835b85e86b"),
}

if __name__ == "__main__":
    import sys

    write_kat(sys.argv[1], sys.argv[2])
