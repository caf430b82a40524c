"""Mode-E golden fixtures, produced by the reference itself (TEST INFRASTRUCTURE ONLY).

Needs oracle/_ref/ (`make -C oracle ref`, this container only).  Writes:

  tests/golden/mode_e.json   per case of mode_e_inputs.CASES: the md5 and size of every output
                             file of the reference CLI run in mode E (`kmerLSH_seeded ... -M E
                             --only`, app/kmerLSH.cc:521-580: AB::WRS, kmer_set.hex, IOFQ::Extracting)
                             and the two differential k-mer counts it prints
  tests/golden/ttest.npz     alglib::studentttest2 (AB::WRS's test, function/funcAB.cc:100) on f32
                             samples as WRS passes them: inputs + the three tails (f64) per case

    python tests/golden/make_golden_e.py
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import mode_e_inputs  # noqa: E402

REF_CLI = os.path.join(ROOT, "oracle", "_ref", "kmerLSH_seeded")
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


def md5(path: str) -> str:
    with open(path, "rb") as f:
        return hashlib.md5(f.read()).hexdigest()


def run_case(case: str) -> dict:
    with tempfile.TemporaryDirectory() as tmp:
        info = mode_e_inputs.write_case(tmp, case)
        env = dict(os.environ, OMP_THREAD_LIMIT="1")
        out = subprocess.run([REF_CLI] + mode_e_inputs.cli_args(case), cwd=tmp, env=env,
                             check=True, capture_output=True, text=True).stdout
        counts = [int(x) for x in re.findall(r"# of differential kmers in group [AB] : (\d+)", out)]
        files = {}
        for prefix, names in (("A", info["samples1"]), ("B", info["samples2"])):
            for nm in names:
                p = os.path.join(tmp, "%s_%s" % (prefix, nm))
                with open(p, "rb") as f:
                    nrec = f.read().count(b"\n@") + (1 if os.path.getsize(p) else 0)
                files["%s_%s" % (prefix, nm)] = dict(md5=md5(p), size=os.path.getsize(p), reads=nrec)
        return dict(args=mode_e_inputs.cli_args(case), kmap=info["kmap"], clusters=info["clusters"],
                    differential=counts, abnormal=out.count("abnormal read entry skipped"),
                    files=files)


def ttest_cases():
    """(n, m, values[count][n+m]) groups: random, shifted, constant, tiny/huge spreads, t < -2."""
    rng = np.random.default_rng(2026)
    out = []
    for n, m in [(4, 4), (3, 2), (5, 5), (32, 32), (1, 1), (1, 3), (2, 1), (7, 12), (0, 3), (3, 0)]:
        cnt = 64
        v = rng.normal(size=(cnt, n + m)).astype(np.float32)
        v[:, :n] += rng.normal(scale=2.0, size=(cnt, 1)).astype(np.float32)
        v[::7] = np.float32(0.5)                       # every value equal: s == 0, equal means
        if n > 0 and m > 0:
            v[3::11, :n] = np.float32(1.0)             # constant groups, different means
            v[3::11, n:] = np.float32(2.0)
            v[5::13] *= np.float32(1e-30)              # tiny spread
            v[6::13] *= np.float32(1e30)               # huge spread
            v[8::9, :n] -= np.float32(40.0)            # very negative t (incomplete-beta branch)
        out.append((n, m, v))
    return out


def main() -> None:
    if not (os.path.exists(REF_CLI) and os.path.exists(HARNESS)):
        sys.exit("build the reference first: make -C oracle ref")
    fix = {case: run_case(case) for case in mode_e_inputs.CASES}
    with open(os.path.join(HERE, "mode_e.json"), "w") as f:
        json.dump(fix, f, indent=1, sort_keys=True)
    arrays = {}
    with tempfile.TemporaryDirectory() as tmp:
        for gi, (n, m, v) in enumerate(ttest_cases()):
            src, dst = os.path.join(tmp, "v.f32"), os.path.join(tmp, "t.f64")
            v.tofile(src)
            subprocess.run([HARNESS, "ttest", src, str(n), str(m), str(v.shape[0]), dst], check=True)
            arrays["v%d" % gi] = v
            arrays["nm%d" % gi] = np.array([n, m], np.int32)
            arrays["t%d" % gi] = np.fromfile(dst, np.float64).reshape(-1, 3)
    np.savez_compressed(os.path.join(HERE, "ttest.npz"), **arrays)
    print("wrote mode_e.json (%d cases), ttest.npz (%d groups)" % (len(fix), len(arrays) // 3))


if __name__ == "__main__":
    main()
