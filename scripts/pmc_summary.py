"""Average rocprofv3 --pmc counters per kernel over dispatches (gpurun_out/pmc/<pass>/c_counter_collection.csv)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(f"{root}/*/c_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    short = k.replace("qlx::qn::", "").replace("qlx::", "")[:90]
    print(short)
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
