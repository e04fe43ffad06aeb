#!/bin/bash
# HBM traffic of the decompress (default) or compress kernel on the bench workload, per the
# MI355X guide's HBM/rocprofv3 recipe: FETCH_SIZE and WRITE_SIZE in separate --pmc passes
# (kernel-trace only, no tracing domains), summarised by tools/pmc_traffic.py.
#   tools/pmc_traffic.sh OUTDIR [generator] [decompress|compress]
set -o pipefail
OUT=$1; GEN=${2:-tiles216}; WHAT=${3:-decompress}
KERNEL=lz4mi_decompress_kernel
[ "$WHAT" = compress ] && KERNEL=lz4mi_compress_gts_kernel
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-include-regex $KERNEL --pmc $pmc -d "$OUT/$pmc" -o pmc \
    --output-format csv -- python tools/microbench.py --what $WHAT --gens $GEN --blocks 4096 --reps 1 > "$OUT/$pmc.log" 2>&1 \
    || { echo "pass $pmc failed"; exit 1; }
done
python tools/pmc_traffic.py "$OUT" "$GEN" "$KERNEL" > "$OUT/pmc_traffic.json" && cat "$OUT/pmc_traffic.json"
