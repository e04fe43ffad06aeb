#!/bin/bash
# FETCH_SIZE calibration for the decoder's read patterns (tools/probe/fetch_calib.hip):
# timing run, then one --pmc pass per counter (kernel trace only).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/fcal; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/probe/fetch_calib > $O/time.log 2>&1 || { echo "timing failed"; exit 1; }
cat $O/time.log
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc $pmc -d $O/$pmc -o pmc --output-format csv -- $R/tools/probe/fetch_calib > $O/$pmc.log 2>&1 || { echo "pass $pmc failed"; exit 1; }
done
find $O -name "*counter_collection*" | head
# (the encoder occupancy A/B in profiles/r02j used a timing-only launch knob, since removed)
