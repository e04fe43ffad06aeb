# tiles216/mix timing of every build under tools/variants/ in one process (the first
# named build is repeated at the end to expose drift).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sweep
V=""; for n in "$@"; do V="$V tools/variants/liblz4mi_$n.so"; done
V="$V tools/variants/liblz4mi_$1.so"
timeout -k 10 500 python tools/microbench.py --gens ${GENS:-tiles216,mix} --blocks 4096 --reps 7 --skip-default --so $V > gpurun_out/sweep/sweep.json 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/sweep/sweep.json; exit 1; }
grep GBps gpurun_out/sweep/sweep.json
