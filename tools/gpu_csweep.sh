# Compress-kernel timing of builds under tools/variants/ in one process (first build repeated last).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sweep
V=""; for n in "$@"; do V="$V tools/variants/liblz4mi_$n.so"; done
V="$V tools/variants/liblz4mi_$1.so"
timeout -k 10 600 python tools/microbench.py --what compress --gens ${GENS:-tiles216,random} --blocks 4096 --reps 3 --skip-default --so $V > gpurun_out/sweep/csweep.json 2>&1 || { echo "csweep failed"; tail -20 gpurun_out/sweep/csweep.json; exit 1; }
grep GBps gpurun_out/sweep/csweep.json
