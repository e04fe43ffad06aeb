"""Per-dispatch instruction counters from a rocprofv3 --pmc CSV (tools/gpu_phase_valu.sh):
one line per dispatch of the decode kernel, in launch order (the microbench runs the default
build first, then the variant: warm-up + timed launch each)."""
import csv
import glob
import json
import sys

rows = {}
for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            rows.setdefault(d, {})[r["Counter_Name"]] = rows.get(d, {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
print(json.dumps([{"dispatch": d, **{k: v for k, v in sorted(c.items())}} for d, c in sorted(rows.items())]))
