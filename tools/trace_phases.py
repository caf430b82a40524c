"""Per-phase critical-path breakdown of the LSH loop from a rocprofv3 kernel trace (CSV).

Iterations are delimited by the projection launch.  For every iteration: the wall span (first
kernel start to the next iteration's projection start), and per phase the span from the phase's
first kernel start to its last kernel end (phases: project, sort, runs, merge, compact), plus the
idle time on the GPU (no kernel running).  Prints totals over head (N >= split) / tail iterations
and the heaviest iterations.

    python tools/trace_phases.py gpurun_out/prof/c2tr/run_kernel_trace.csv [--skip 1]
"""
import argparse
import csv
from collections import defaultdict

PHASES = (
    ("project", ("k_project",)),
    ("sort", ("k_radix", "k_scan", "k_sort")),
    ("runs", ("k_runs", "k_classify")),
    ("merge", ("k_merge",)),
    ("compact", ("k_compact",)),
)


def phase_of(name):
    for p, keys in PHASES:
        if any(k in name for k in keys):
            return p
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=1, help="leading iterations to drop (init pass)")
    ap.add_argument("--top", type=int, default=8)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                 r.get("Grid_Size_X", ""), r.get("Stream_Id", "")) for r in rows)
    its, cur = [], None
    for k in ks:
        if "k_project" in k[2] and "fix" not in k[2]:
            cur = []
            its.append(cur)
        if cur is not None:
            cur.append(k)
    its = its[args.skip:]
    recs = []
    for idx, it in enumerate(its):
        t0 = it[0][0]
        t1 = its[idx + 1][0][0] if idx + 1 < len(its) else max(b for _, b, *_ in it)
        span = defaultdict(lambda: [None, None])
        busy = []
        for a, b, n, g, s in it:
            p = phase_of(n)
            sp = span[p]
            sp[0] = a if sp[0] is None else min(sp[0], a)
            sp[1] = b if sp[1] is None else max(sp[1], b)
            busy.append((a, b))
        busy.sort()
        covered, ca, cb = 0, None, None
        for a, b in busy:
            if ca is None or a > cb:
                if ca is not None:
                    covered += cb - ca
                ca, cb = a, b
            else:
                cb = max(cb, b)
        covered += cb - ca
        rec = {"it": idx, "wall": (t1 - t0) / 1e3, "idle": (t1 - t0 - covered) / 1e3,
               "tail": any("k_merge_tail" in k[2] for k in it)}
        for p, _ in PHASES + (("other", ()),):
            a, b = span[p]
            rec[p] = (b - a) / 1e3 if a is not None else 0.0
        recs.append(rec)
    cols = [p for p, _ in PHASES] + ["other", "idle", "wall"]
    print(f"{'iterations':>22} " + " ".join(f"{c:>9}" for c in cols) + "   (ms, phase spans)")
    head = [r for r in recs if not r["tail"]]  # the tail: iterations merged by k_merge_tail
    tail = [r for r in recs if r["tail"]]
    for label, sel in (("all", recs), (f"head ({len(head)})", head), (f"tail ({len(tail)})", tail)):
        tot = {c: sum(r[c] for r in sel) / 1e3 for c in cols}
        print(f"{label:>22} " + " ".join(f"{tot[c]:9.2f}" for c in cols))
    print(f"\nheaviest {args.top} iterations (us):")
    for r in sorted(recs, key=lambda r: -r["wall"])[: args.top]:
        print(f"  it {r['it']:4d} " + " ".join(f"{c}={r[c]:.0f}" for c in cols))
    for probe in (0, 1, 50, 100, 200, 300, 450):
        if probe < len(recs):
            r = recs[probe]
            print(f"  it {probe:4d} " + " ".join(f"{c}={r[c]:.0f}" for c in cols))


if __name__ == "__main__":
    main()
