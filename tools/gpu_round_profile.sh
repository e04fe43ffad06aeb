# Round-end measurement set: full bench line, rocprof kernel stats of the same command,
# HBM traffic (tiles216 single-pass kernel; repetitive ring decoder).
set -o pipefail
TAG=${1:-r01f}
bash tools/run_bench_profile.sh $TAG || exit 1
O=gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-include-regex "ring_decode|token_map" --pmc $pmc -d "$O/ring_$pmc" -o pmc \
    --output-format csv -- python tools/microbench.py --gens repetitive --blocks 4096 --reps 1 > "$O/ring_$pmc.log" 2>&1 \
    || { echo "ring pass $pmc failed"; exit 1; }
done
python tools/pmc_summary.py_dummy 2>/dev/null; for f in $O/ring_FETCH_SIZE $O/ring_WRITE_SIZE; do cat $(find $f -name "*counter_collection.csv") | cut -d, -f1-30 | head -5; done > $O/ring_pmc.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rep -o run --output-format csv -- python tools/microbench.py --gens repetitive,random --blocks 4096 --reps 3 > $O/prof_rep.log 2>&1 || { echo "rep stats failed"; exit 1; }
echo ok
