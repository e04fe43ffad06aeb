#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (one dir per pass): mean counter value per dispatch of each kernel."""
import collections, csv, glob, json, sys
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in acc.items():
    out[k] = {c: (sum(v) / len(v)) for c, v in cs.items()}
print(json.dumps(out, indent=1))
