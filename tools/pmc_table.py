"""Per-kernel mean of every counter collected under <dir>/p*/run_counter_collection.csv."""
import csv
import glob
import sys
from collections import defaultdict

d = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(d.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    if "cv::" not in k:
        continue
    print(k.split("(")[0])
    for c, v in sorted(cs.items()):
        print(f"   {c:36s} {sum(v) / len(v):16.0f}")
