#!/bin/bash
# Round-end measurement: bench line, kernel-trace stats of the same command,
# HBM traffic counters. Outputs under gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-r01}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --extra 0 --cpu-baseline 0 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*stats*" | head
tools/pmc_traffic.sh $O/pmc tiles216 > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
cat $O/pmc/pmc_traffic.json
