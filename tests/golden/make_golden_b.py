"""Mode-B golden fixtures, produced by the reference itself (TEST INFRASTRUCTURE ONLY).

Needs oracle/_ref/kmerLSH_seeded (`make -C oracle ref`, this container only).  For every case of
kmc_inputs.CASES and kmc_inputs.BIG_CASES["bl_fill"] the reference CLI runs `-M B --only -T 1`
(buildKHtable with kmc = false, io/ioHT.cc:83-199) on the synthesized KMC databases;
tests/golden/mode_b.json keeps kmer_count.log verbatim, the md5 of the reference's kmer_set.hex
and kmer_count.bin (rows in its libcuckoo table order), and an order-free digest of the rows (md5
over the rows sorted by k-mer, each row = the 8-byte k-mer + its d uint16 counts).  bl_fill loads
the table's 2^16 8-slot buckets to 95.6 % (long cuckoo paths, no growth).  A case past that
("bl_grow") is not kept: the reference doubles its table by re-inserting from
hardware_concurrency() threads, and two runs of it wrote different row orders here.

    python tests/golden/make_golden_b.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import kmc_inputs  # noqa: E402
import klsh_oracle_b as ob  # noqa: E402

REF_CLI = os.path.join(ROOT, "oracle", "_ref", "kmerLSH_seeded")


def row_digest(reps, counts) -> str:
    import hashlib

    import numpy as np

    idx = np.argsort(np.asarray(reps, np.uint64), kind="stable")
    h = hashlib.md5()
    for i in idx:
        h.update(int(reps[i]).to_bytes(8, "little"))
        h.update(np.ascontiguousarray(counts[:, i], np.uint16).tobytes())
    return h.hexdigest()


def main() -> None:
    if not os.path.exists(REF_CLI):
        sys.exit("build the reference first: make -C oracle ref")
    import hashlib

    out = {}
    for case in list(kmc_inputs.CASES) + ["bl_fill"]:
        big = case in kmc_inputs.BIG_CASES
        with tempfile.TemporaryDirectory() as tmp:
            info = (kmc_inputs.write_big_case if big else kmc_inputs.write_case)(tmp, case)
            args = kmc_inputs.big_cli_args(case) if big else kmc_inputs.cli_args(case)
            subprocess.run([REF_CLI] + args, cwd=tmp, check=True,
                           capture_output=True, env=dict(os.environ, OMP_THREAD_LIMIT="1"))
            reps, counts, log = ob.read_outputs(tmp, info["d"])
            md5f = lambda n: hashlib.md5(open(os.path.join(tmp, n), "rb").read()).hexdigest()  # noqa: E731
            out[case] = dict(kmap=int(len(reps)), log=log, rows_md5=row_digest(reps, counts),
                             hex_md5=md5f("kmer_set.hex"), bin_md5=md5f("kmer_count.bin"),
                             saturated=int((counts == 65535).sum()), has_zero_kmer=bool((reps == 0).any()))
    with open(os.path.join(HERE, "mode_b.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote mode_b.json:", {c: v["kmap"] for c, v in out.items()})


if __name__ == "__main__":
    main()
