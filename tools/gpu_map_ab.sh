#!/bin/bash
# pass-1 (token map) kernel time of variant builds, bitmap mode, tiles216:
#   tools/gpu_map_ab.sh so1 so2 ...   (rocprofv3 kernel stats per variant)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mapab
for so in "$@"; do
  n=$(basename $so .so)
  LZ4MI_BITMAP=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mapab/$n -o run --output-format csv -- \
    python tools/microbench.py --gens tiles216 --blocks 4096 --reps 2 --so $so --skip-default > gpurun_out/mapab/$n.log 2>&1 \
    || { tail gpurun_out/mapab/$n.log; exit 1; }
  echo "$n: $(grep tiles216 gpurun_out/mapab/$n.log)"
  grep -h "token_map\|bm_kernel" $(find gpurun_out/mapab/$n -name "*kernel_stats.csv") | cut -d, -f1-4
done
