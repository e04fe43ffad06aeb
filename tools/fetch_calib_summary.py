#!/usr/bin/env python3
"""Summarise tools/gpu_fetch_calib.sh: per probe kernel, FETCH_SIZE and WRITE_SIZE
(KiB -> bytes, raw, uncorrected) against the bytes the kernel reads by
construction (tools/probe/fetch_calib.hip), i.e. the counter factor per access
pattern. Second-rep dispatches only (the first rep warms the code object).
  python tools/fetch_calib_summary.py gpurun_out/fcal > profiles/<tag>/fetch_calib.json"""
import csv, glob, json, sys

root = sys.argv[1]
GiB = 1 << 30
known = {"k_stream": 2 * GiB, "k_lines": 2 * GiB, "k_half": 1 * GiB, "k_piece": GiB // 4,
         "k_decoder": 1024 * ((4 << 20) - 36864)}
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{root}/{c}/**/pmc_counter_collection.csv", recursive=True):
        rows = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != c:
                continue
            k = next((k for k in known if k in r["Kernel_Name"]), None)
            if k:
                rows.setdefault(k, []).append(float(r["Counter_Value"]) * 1024)
        for k, v in rows.items():
            out.setdefault(k, {"known_read_bytes": known[k]})[c + "_bytes"] = v[-1]
for k, d in out.items():
    if "FETCH_SIZE_bytes" in d:
        d["fetch_over_known"] = round(d["FETCH_SIZE_bytes"] / d["known_read_bytes"], 4)
times = {}
try:
    for line in open(f"{root}/time.log"):
        p = line.split()
        if len(p) > 6 and p[0] == "rep" and p[1] == "1":
            times[p[2].split("(")[0]] = float(p[p.index("ms") - 1])
except OSError:
    pass
for k, ms in times.items():
    out.setdefault(k, {"known_read_bytes": known.get(k)})["ms"] = ms
print(json.dumps(out, indent=1))
