# Phase profile of the ring decoder + rocprof kernel stats of the default build.
set -o pipefail
O=gpurun_out/${1:-rp}
mkdir -p $O
timeout -k 10 200 python tools/ring_prof.py --so tools/variants/liblz4mi_ringprof.so --gen tiles216 > $O/prof_tiles.txt 2>&1 || { echo fail; tail -20 $O/prof_tiles.txt; exit 1; }
cat $O/prof_tiles.txt
timeout -k 10 200 python tools/ring_prof.py --so tools/variants/liblz4mi_ringprof.so --gen random > $O/prof_random.txt 2>&1 || { echo fail; tail -20 $O/prof_random.txt; exit 1; }
cat $O/prof_random.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 3 > $O/rocprof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/rocprof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 $f | head -12
