"""Summarise a rocprofv3 --pmc CSV directory: per kernel name, mean of each counter."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
agg = defaultdict(lambda: defaultdict(list))
for f in files:
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "?")[:48]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("GRBM_GUI_ACTIVE", [0]))):
    n = max(len(v) for v in cs.values())
    print("{:48s} n={:6d} ".format(name, n) + " ".join("{}={:.4g}".format(k, sum(v) / len(v)) for k, v in sorted(cs.items())))
