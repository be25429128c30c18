"""Summarise scripts/prof_quick.sh output: per kernel calls, average us (rocprofv3 --stats) and average HBM
fetch per dispatch (FETCH_SIZE x 2, the gfx950 correction of MI355X_MICROARCH.md)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
stats = glob.glob(os.path.join(root, "stats", "**", "*kernel_stats.csv"), recursive=True)
fetch = glob.glob(os.path.join(root, "fetch", "**", "*counter_collection.csv"), recursive=True)
fb = defaultdict(list)
for f in fetch:
    for r in csv.DictReader(open(f)):
        if r.get("Counter_Name") == "FETCH_SIZE":
            fb[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024 * 2)


def short(n):
    n = n.split("(")[0]
    return n[-60:]


rows = []
for f in stats:
    for r in csv.DictReader(open(f)):
        name = r["Name"]
        v = fb.get(name, [])
        rows.append((float(r["TotalDurationNs"]), short(name), int(r["Calls"]), float(r["AverageNs"]) / 1e3,
                     (sum(v) / len(v) / 1e6) if v else float("nan")))
rows.sort(reverse=True)
print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>9s} {'fetch_MB':>9s} {'total_ms':>9s}")
for tot, n, c, avg, mb in rows:
    print(f"{n:60s} {c:6d} {avg:9.2f} {mb:9.2f} {tot / 1e6:9.3f}")
