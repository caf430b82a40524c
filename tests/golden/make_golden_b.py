"""Mode-B golden fixtures, produced by the reference itself (TEST INFRASTRUCTURE ONLY).

Needs oracle/_ref/kmerLSH_seeded (`make -C oracle ref`, this container only).  For every case of
kmc_inputs.CASES the reference CLI runs `-M B --only` (buildKHtable with kmc = false, io/ioHT.cc:
83-199) on the synthesized KMC databases; tests/golden/mode_b.json keeps kmer_count.log verbatim
and an order-free digest of the rows (the reference's row order is its libcuckoo table's):
md5 over the rows sorted by k-mer, each row = the 8-byte k-mer + its d uint16 counts.

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
    out = {}
    for case in kmc_inputs.CASES:
        with tempfile.TemporaryDirectory() as tmp:
            info = kmc_inputs.write_case(tmp, case)
            subprocess.run([REF_CLI] + kmc_inputs.cli_args(case), cwd=tmp, check=True,
                           capture_output=True, env=dict(os.environ, OMP_THREAD_LIMIT="1"))
            reps, counts, log = ob.read_outputs(tmp, info["d"])
            out[case] = dict(kmap=int(len(reps)), log=log, rows_md5=row_digest(reps, counts),
                             saturated=int((counts == 65535).sum()), has_zero_kmer=bool((reps == 0).any()))
    with open(os.path.join(HERE, "mode_b.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote mode_b.json:", {c: v["kmap"] for c, v in out.items()})


if __name__ == "__main__":
    main()
