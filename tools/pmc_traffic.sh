#!/bin/bash
# HBM traffic of the decompress kernel on the bench workload, per the MI355X
# guide's HBM/rocprofv3 recipe: FETCH_SIZE and WRITE_SIZE in separate --pmc
# passes (kernel-trace only, no tracing domains), then summarised into
# profiles/pmc_traffic.json by tools/pmc_traffic.py.
#   tools/pmc_traffic.sh OUTDIR [generator]
set -o pipefail
OUT=$1; GEN=${2:-tiles216}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-include-regex lz4mi_decompress_kernel --pmc $pmc -d "$OUT/$pmc" -o pmc \
    --output-format csv -- python tools/microbench.py --gens $GEN --blocks 4096 --reps 1 > "$OUT/$pmc.log" 2>&1 \
    || { echo "pass $pmc failed"; exit 1; }
done
python tools/pmc_traffic.py "$OUT" "$GEN" > "$OUT/pmc_traffic.json" && cat "$OUT/pmc_traffic.json"
