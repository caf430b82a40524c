"""Print the kernel timeline of chosen LSH iterations from a rocprofv3 kernel trace (CSV)."""
import csv
import sys

path = sys.argv[1]
which = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 100, 400]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
its, cur = [], None
for r in rows:
    n = r["Kernel_Name"]
    if "k_project" in n:
        cur = []
        its.append(cur)
    if cur is not None:
        cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r["Grid_Size_X"], r["Stream_Id"]))
its = its[1:]  # the init pass
for i in which:
    k = its[i]
    t0 = k[0][0]
    print(f"iteration {i}: {(max(b for _, b, *_ in k) - t0) / 1e3:.1f} us")
    for a, b, n, g, s in k:
        print(f"   s{s} {(a - t0) / 1e3:8.1f} {(b - a) / 1e3:7.1f}  grid {g:>8} {n.split('(')[0][:70]}")
