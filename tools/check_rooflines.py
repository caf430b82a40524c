"""Recompute every kernel-class roofline fraction of a bench line from the committed rocprofv3
kernel trace of the same workload (profiles/<tag>_<cfg>_class_times.json, made by
tools/pmc_summary.py) and report how far the bench's own launch times are from rocprof's.

  python tools/check_rooflines.py r05 [c2]   -> profiles/<tag>_<cfg>_roofline_check.txt

The bench lines checked are the one printed inside the rocprofv3 run (<tag>_<cfg>_stats.log, same
process as the trace) and the separate bench run (<tag>_<cfg>_bench.log).  frac_rocprof = the
bench's algorithmic bytes per class launch / rocprof's average class-launch duration / 8 TB/s.
Span classes (several dependent launches: sort, runs, compact) are the sum of their dispatch
durations in rocprof and first-start -> last-end in the bench, so the bench's includes the gaps.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def bench_line(path):
    with open(path) as f:
        lines = [ln for ln in f if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r05"
    cfg = sys.argv[2] if len(sys.argv) > 2 else "c2"
    ct = json.load(open(os.path.join(PROF, f"{tag}_{cfg}_class_times.json")))["classes"]
    out = []
    worst = None
    for kind in ("stats", "bench"):
        path = os.path.join(PROF, f"{tag}_{cfg}_{kind}.log")
        if not os.path.exists(path):
            continue
        line = bench_line(path)
        if not line:
            continue
        out.append(f"== {os.path.basename(path)}: value {line['value']:.4g}, "
                   f"{line['ms_per_step']:.2f} ms/step")
        out.append(f"{'class':8s} {'kernel':42s} {'timing':10s} {'bench_ms':>9s} {'rocprof_ms':>10s}"
                   f" {'diff':>7s} {'frac':>8s} {'frac_rocprof':>12s}")
        for k in line["roofline"]["kernels"]:
            c = k["class"]
            r = ct.get(c)
            if not r:
                continue
            ours, theirs = k["avg_launch_ms"], r["avg_launch_ms"]
            diff = ours / theirs - 1.0
            fr = k["bytes_per_launch"] / (theirs * 1e-3) / 1e9 / k["peak"]
            span = r["dispatches"] != r["class_launches"]
            if kind == "stats" and not span and not k.get("overlapped"):
                worst = max(worst or 0.0, abs(diff))
            out.append(f"{c:8s} {k['kernel'][:42]:42s} {k.get('timing', ''):10s} {ours:9.4f} "
                       f"{theirs:10.4f} {diff:+7.1%} {k['frac']:8.4f} {fr:12.4f}"
                       + ("  (span)" if span else "") + ("  (overlapped)" if k.get("overlapped")
                                                          else ""))
        h = line["roofline"]
        out.append(f"headline: {h['kernel']} frac {h['frac']} (rocprof: "
                   f"{h['bytes_per_launch'] / (ct[h['class']]['avg_launch_ms'] * 1e-3) / 1e9 / h['peak']:.4f})")
    out.append("largest |bench - rocprof| over the single-dispatch classes that run alone, same "
               "run: " + (f"{worst:.1%}" if worst is not None else "n/a (none at this d)"))
    text = "\n".join(out) + "\n"
    with open(os.path.join(PROF, f"{tag}_{cfg}_roofline_check.txt"), "w") as f:
        f.write(text)
    print(text)


if __name__ == "__main__":
    main()
