"""Fold the rocprofv3 outputs of tools/collect_profiles.sh into profiles/ (round-named files) and
profiles/pmc_summary.json (HBM bytes per projection launch: FETCH_SIZE x 2 + WRITE_SIZE, KB -> B,
the gfx950 correction of MI355X_MICROARCH.md §HBM; averaged over the main loop's launches)."""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "gpurun_out", "prof")
dst = os.path.join(ROOT, "profiles")
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"


def one(pattern):
    m = glob.glob(os.path.join(src, pattern), recursive=True)
    return m[0] if m else None


def stats_txt(csv_path, txt_path):
    rows = list(csv.DictReader(open(csv_path)))
    tot = sum(float(x["TotalDurationNs"]) for x in rows)
    with open(txt_path, "w") as f:
        for x in rows:
            f.write(f"{x['Name'][:70]:70s} calls={int(x['Calls']):6d} total_ms={float(x['TotalDurationNs'])/1e6:9.2f} "
                    f"avg_us={float(x['AverageNs'])/1e3:9.2f} pct={float(x['Percentage']):6.2f}\n")
        f.write(f"total kernel time {tot/1e6:.2f} ms\n")


for cfg in ("c2", "c4", "c5"):
    s = one(f"{cfg}_stats/**/run_kernel_stats.csv")
    if s:
        shutil.copy(s, os.path.join(dst, f"{tag}_{cfg}_kernel_stats.csv"))
        stats_txt(s, os.path.join(dst, f"{tag}_{cfg}_kernel_stats.txt"))
for cfg in ("c2", "c4", "c5"):
    b = os.path.join(src, f"{cfg}_bench.log")
    if os.path.exists(b):
        shutil.copy(b, os.path.join(dst, f"{tag}_{cfg}_bench.log"))

summary = {}
# (kernel key, regex used by collect_profiles.sh, launches to keep: the main loop's — the init
# pass's launch comes first)
for key, keep in (("k_project", 500), ("k_merge_small", None), ("k_small_screen", None)):
    vals = {}
    for kind, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        p = one(f"c2_{kind}_{key}/**/run_counter_collection.csv") or (
            one(f"c2_{kind}/**/run_counter_collection.csv") if key == "k_project" else None)
        if not p:
            continue
        shutil.copy(p, os.path.join(dst, f"{tag}_c2_pmc_{kind}_{key}.csv"))
        rows = [r for r in csv.DictReader(open(p)) if r["Counter_Name"] == counter]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        rows = rows[-keep:] if keep else rows[1:]
        vals[kind] = (sum(float(r["Counter_Value"]) for r in rows) * 1024.0 / len(rows), len(rows),
                      rows[0]["Kernel_Name"].split("(")[0])
    if "fetch" in vals and "write" in vals:
        f, n, name = vals["fetch"]
        w, _, _ = vals["write"]
        summary.setdefault("c2", {})[key] = {
            "kernel": name, "launches": n,
            "raw_fetch_bytes_per_launch": f, "raw_write_bytes_per_launch": w,
            "hbm_bytes_per_launch": 2 * f + w,
            "correction": "FETCH_SIZE x2 (gfx950 counts 16-B/lane reads at half, MI355X_MICROARCH.md §HBM); WRITE_SIZE as read",
            "note": "FETCH_SIZE counts Infinity-Cache hits too; the late iterations (<1M rows) are MALL-resident",
            "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, --kernel-include-regex {key}), bench.py --steps 1 --warmup 0, round {tag}",
        }
if summary:
    json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
