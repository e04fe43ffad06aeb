"""Summarise tools/phase_counts.sh: per-phase instruction counts of the decoder, per sequence and per
1 KiB chunk of compressed input, as differences between the cumulative ablation builds.
  python tools/phase_counts.py OUTDIR"""
import csv, glob, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
O = sys.argv[1]
ORDER = [("abl3", "stage + next-token table"), ("abl2", "jump tables + walks + certification"),
         ("abl1", "sequence table + checks"), ("abl6", "output round 1 (map, literals, remap, pieces)"),
         ("default", "output rounds 2+, cut sequence")]
ROUND1 = [("abl1", "through the sequence table"), ("abl7c", "round 1: literals, match planning"),
          ("abl7b", "round 1: output -> sequence map"), ("abl7", "round 1: remap of in-chunk sources"),
          ("abl6", "round 1: match copies (piece pipeline)"), ("default", "rounds 2+, cut sequence")]
SEQ_PER_BLOCK = 61030.0     # tiles216 4 MiB, oracle parse (seed 1: 61 034, seed 2: 61 019)
COMP_PER_BLOCK = 526e3      # compressed bytes per block (bench: 7.974:1)


def counts(v):
    f = glob.glob(os.path.join(O, v, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for r in csv.DictReader(open(f[0])):
        per.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
    d = list(per.values())[-1]    # the timed launch (the first is the warm-up; both equal)
    return d


if len(sys.argv) > 2 and sys.argv[2] == "round1":
    ORDER = ROUND1
res = {v: counts(v) for v, _ in ORDER}
times = {}
for line in open(os.path.join(O, "times.log")):
    p = line.split(" ", 2)
    if len(p) == 3 and p[0] == "tiles216":
        times[p[1].replace("liblz4mi_", "").replace(".so", "")] = json.loads(p[2])["ms"]
out = {"workload": "4096 x 4 MiB tiles216 decode, one PMC pass per build", "seq_per_block": SEQ_PER_BLOCK, "phases": []}
prev = None
for v, what in ORDER:
    c = res[v]
    waves = c["SQ_WAVES"]
    row = {"build": v, "phase": what, "ms": times.get(v)}
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
        cum = c[k] / waves / SEQ_PER_BLOCK
        row[k.replace("SQ_INSTS_", "") + "_per_seq_cum"] = round(cum, 2)
        row[k.replace("SQ_INSTS_", "") + "_per_seq"] = round(cum - (prev[k] / prev["SQ_WAVES"] / SEQ_PER_BLOCK if prev else 0), 2)
    prev = c
    out["phases"].append(row)
print(json.dumps(out, indent=1))
