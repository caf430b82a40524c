"""The sharded loop's decomposition, on CPU with gloo at world sizes 2 and 3: key-range ownership
by row midpoint + exchange in source-rank order + per-range stable bucket order reproduce the
single-process Cluster() exactly (tests/shard_model_worker.py; the GPU engine's own sharded
loop is checked against the single-GPU engine in tests/test_gpu_sharded.py)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from test_distributed import free_port

CFG = {"seed": 5, "rng_seed": 777, "n": 3000, "d": 8, "iters": 8, "min_sim": 0.8, "noise": 0.05}


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_model_matches_single(oracle, tmp_path, world):
    out = tmp_path / "model.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "shard_model_worker.py")]
    env = dict(os.environ, OMP_NUM_THREADS="1", KLSH_MODEL_CFG=json.dumps(CFG),
               KLSH_MODEL_OUT=str(out))
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300, env=env)
    got = json.loads(out.read_text())

    rng = np.random.default_rng(CFG["seed"])
    n, d = CFG["n"], CFG["d"]
    centers = rng.normal(0, 1, (max(n // 20, 1), d)).astype(np.float32)
    rows = (centers[rng.integers(0, centers.shape[0], n)] +
            rng.normal(0, CFG["noise"], (n, d))).astype(np.float32)
    ref, off, ids, trace, counter = oracle.cluster(rows, CFG["min_sim"], CFG["iters"], 1_000_000,
                                                   seed=CFG["rng_seed"])
    assert len(trace) == CFG["iters"] and ref.shape[0] < n  # merges happened
    assert got["counter"] == counter
    assert np.array_equal(np.array(got["rows"], np.uint32).reshape(-1, d), ref.view(np.uint32))
    want = [ids[int(off[j]):int(off[j + 1])].tolist() for j in range(ref.shape[0])]
    assert got["ids"] == want
