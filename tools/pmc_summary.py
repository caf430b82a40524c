"""Fold the rocprofv3 outputs of tools/collect_profiles.sh into profiles/ (round-named files):

  <tag>_<cfg>_kernel_stats.{csv,txt}   rocprofv3 --stats of one bench step
  <tag>_<cfg>_class_times.json         the main loop's launches of the same run grouped by bench.py
                                       kernel class (dispatch count, summed and average duration)
  <tag>_c2_pmc_{fetch,write}_<class>.csv  the counter passes
  pmc_summary.json                     HBM bytes per class launch of the C2 main loop: FETCH_SIZE x 2
                                       + WRITE_SIZE, KB -> B (the gfx950 correction of
                                       MI355X_MICROARCH.md §HBM)

The main loop is told apart from the init pass (app/kmerLSH.cc:323, one iteration on the same
rows) by the projection: every counter pass also collects k_project, and the loop starts at its
second dispatch.  A class launch is what bench.py counts as one (klsh_stats.kern): one dispatch
for k_merge_small / k_merge_tail / k_small_screen, one iteration for the span classes (sort: the
hist/dscan/scatter passes; runs: k_runs_* at the head, k_tail_local in the tail; compact).
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "gpurun_out", "prof")
dst = os.path.join(ROOT, "profiles")
tag = sys.argv[1] if len(sys.argv) > 1 else "r05"

# bench.py kernel class -> kernel-name regex (d > 64: the wide kernels; big192 and big384 share
# k_merge_big_wide<384,256,32> there, listed under big384).  A class launch is one dispatch when the
# class is one kernel, else one iteration (the span classes, the wide small-run chain).
CLASSES = {
    "project": r"k_project",
    "sort": r"k_sort_",
    "runs": r"k_runs_|k_tail_local",
    "screen": r"k_small_screen",
    "small": r"k_merge_small|k_merge_group_wide",
    "tail": r"k_merge_tail",
    "big128": r"k_merge_big<\d+, 128|k_merge_big_wide<128",
    "big192": r"k_merge_big<\d+, 192",
    "big384": r"k_merge_big<\d+, 384|k_merge_big_wide<384",
    "big896": r"k_merge_big<\d+, 896|k_merge_big_wide<896",
    "huge": r"k_merge_huge|k_merge_long",
    "compact": r"k_compact",
}
# the counter passes (collect_profiles.sh runs one FETCH_SIZE and one WRITE_SIZE pass each; the
# merge classes, C4 and C5 through its "pmcx" passes)
PMC_CLASSES = {
    "c2": ("project", "screen", "small", "sort", "tail", "runs", "compact", "big128", "big192",
           "big384", "big896"),
    "c4": ("big384", "huge"),
    "c5": ("project", "small", "big384"),
}


def one(pattern):
    m = glob.glob(os.path.join(src, pattern), recursive=True)
    return m[0] if m else None


def short(name):
    return re.sub(r"^void ", "", name.split("(")[0])


def stats_txt(csv_path, txt_path):
    rows = list(csv.DictReader(open(csv_path)))
    tot = sum(float(x["TotalDurationNs"]) for x in rows)
    with open(txt_path, "w") as f:
        for x in rows:
            f.write(f"{x['Name'][:70]:70s} calls={int(x['Calls']):6d} total_ms={float(x['TotalDurationNs'])/1e6:9.2f} "
                    f"avg_us={float(x['AverageNs'])/1e3:9.2f} pct={float(x['Percentage']):6.2f}\n")
        f.write(f"total kernel time {tot/1e6:.2f} ms\n")


def is_iter(r):
    """One per iteration: the projection (not its wide-row fix-up launch, k_project_fix)."""
    return "k_project" in r["Kernel_Name"] and "k_project_fix" not in r["Kernel_Name"]


def loop_start(rows):
    """Dispatch id of the main loop's first projection (the second projection dispatch)."""
    proj = sorted(int(r["Dispatch_Id"]) for r in rows if is_iter(r))
    return proj[1] if len(proj) > 1 else 0


def class_times(trace_csv):
    rows = list(csv.DictReader(open(trace_csv)))
    start = loop_start(rows)
    loop = [r for r in rows if int(r["Dispatch_Id"]) >= start]
    iters = sum(1 for r in loop if is_iter(r))
    out = {"iterations": iters, "source": f"rocprofv3 --kernel-trace --stats, bench.py --steps 1 "
           f"--warmup 0, main-loop dispatches (from the second k_project), round {tag}",
           "classes": {}}
    for c, rx in CLASSES.items():
        sel = [r for r in loop if re.search(rx, r["Kernel_Name"])]
        if not sel:
            continue
        ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel)
        per_dispatch = len({r["Kernel_Name"] for r in sel}) == 1
        launches = len(sel) if per_dispatch else iters
        out["classes"][c] = {
            "kernels": sorted({short(r["Kernel_Name"]) for r in sel}), "dispatches": len(sel),
            "class_launches": launches, "sum_ms": ns / 1e6, "avg_launch_ms": ns / 1e6 / launches,
            "note": "sum of the dispatch durations (a span class's gaps between its dependent "
                    "launches are not in it)" if not per_dispatch else "per dispatch"}
    return out


for cfg in ("c2", "c4", "c5"):
    s = one(f"{cfg}_stats/**/run_kernel_stats.csv")
    if s:
        shutil.copy(s, os.path.join(dst, f"{tag}_{cfg}_kernel_stats.csv"))
        stats_txt(s, os.path.join(dst, f"{tag}_{cfg}_kernel_stats.txt"))
    t = one(f"{cfg}_stats/**/run_kernel_trace.csv")
    if t:
        json.dump(class_times(t), open(os.path.join(dst, f"{tag}_{cfg}_class_times.json"), "w"),
                  indent=1)
    for kind in ("bench", "stats"):
        b = os.path.join(src, f"{cfg}_{kind}.log")
        if os.path.exists(b):
            shutil.copy(b, os.path.join(dst, f"{tag}_{cfg}_{kind}.log"))

summary = {}
old_path = os.path.join(dst, "pmc_summary.json")
if os.path.exists(old_path):  # classes not collected this time keep their earlier entries
    summary = json.load(open(old_path))
for cfg, classes in PMC_CLASSES.items():
    for c in classes:
        rx = CLASSES[c]
        vals = {}
        for kind, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
            p = one(f"{cfg}_{kind}_{c}/**/run_counter_collection.csv")
            if not p:
                continue
            shutil.copy(p, os.path.join(dst, f"{tag}_{cfg}_pmc_{kind}_{c}.csv"))
            rows = [r for r in csv.DictReader(open(p)) if r["Counter_Name"] == counter]
            start = loop_start(rows)
            iters = sum(1 for r in rows if is_iter(r) and int(r["Dispatch_Id"]) >= start)
            sel = [r for r in rows if int(r["Dispatch_Id"]) >= start and re.search(rx, r["Kernel_Name"])]
            launches = len(sel) if len({r["Kernel_Name"] for r in sel}) == 1 else iters
            vals[kind] = (sum(float(r["Counter_Value"]) for r in sel) * 1024.0, launches, len(sel),
                          sorted({short(r["Kernel_Name"]) for r in sel}))
        if "fetch" in vals and "write" in vals and vals["fetch"][1]:
            f, n, nd, names = vals["fetch"]
            w = vals["write"][0]
            note = ("main-loop dispatches only; FETCH_SIZE counts Infinity-Cache hits too; the "
                    "late iterations (<1M rows) are MALL-resident")
            if cfg == "c5" and c == "big384":
                note += ("; k_merge_big_wide<384,256,32> runs both the 129..192- and the "
                         "193..384-row class (one dispatch each per iteration): their average")
            summary.setdefault(cfg, {})[c] = {
                "kernels": names, "launches": n, "dispatches": nd,
                "raw_fetch_bytes_per_launch": f / n, "raw_write_bytes_per_launch": w / n,
                "hbm_bytes_per_launch": (2 * f + w) / n,
                "correction": "FETCH_SIZE x2 (gfx950 counts 16-B/lane reads at half, "
                              "MI355X_MICROARCH.md §HBM); WRITE_SIZE as read",
                "note": note,
                "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, "
                          f"--kernel-include-regex '{rx}|k_project'), bench.py --config {cfg} "
                          f"--steps 1 --warmup 0, round {tag}",
            }
if summary:
    json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
