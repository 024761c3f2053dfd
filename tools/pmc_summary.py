"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch of the kernels matching a name."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "vrc_march"
agg = collections.defaultdict(list)
for fn in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: sum(v) / len(v) for k, v in sorted(agg.items())}
for k, v in res.items():
    print(f"{k:34s} {v:16.1f}  (n={len(agg[k])})")
print(json.dumps(res))
