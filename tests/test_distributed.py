"""bench.py's multi-rank path with world_size 2 on CPU (gloo): every rank reports the same,
maximal elapsed time (the slower rank's), and all K steps ran on every rank."""
import json
import os
import socket
import subprocess
import sys

from conftest import ROOT


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_timing(tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "dist_worker.py")]
    env = dict(os.environ, OMP_NUM_THREADS="1", KLSH_DIST_OUT=str(tmp_path))
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300, env=env)
    recs = [json.loads(p.read_text()) for p in sorted(tmp_path.glob("rank*.json"))]
    assert sorted(r["rank"] for r in recs) == [0, 1]
    e = {r["rank"]: r["elapsed"] for r in recs}
    assert e[0] == e[1]                 # max over ranks
    assert e[0] >= 3 * 0.1 * 0.95       # rank 1's three 0.1 s steps
    assert all(r["res"] == [r["rank"]] * 3 for r in recs)
