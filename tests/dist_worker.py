"""Multi-rank plumbing of bench.py on CPU (gloo): barrier + max-over-ranks timing."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

world, rank, local = bench.dist_setup()
delay = 0.05 * (rank + 1)  # rank 1 is slower: the max must be rank 1's time
elapsed, res = bench.timed(lambda: time.sleep(delay) or rank, steps=3, warmup=1, world=world,
                           local=local, sync=lambda _l: None)
# one file per rank: two ranks printing to one pipe can interleave their lines
with open(os.path.join(os.environ["KLSH_DIST_OUT"], f"rank{rank}.json"), "w") as f:
    json.dump({"rank": rank, "world": world, "elapsed": elapsed, "res": res}, f)
