# Small-batch latency: single-pass vs ring decoder at 64 / 512 / 1024 blocks.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/small
for nb in 64 512 1024; do
  for m in single ring; do
    LZ4MI_DECODER=$m timeout -k 10 300 python tools/microbench.py --gens tiles216,repetitive,random,mix --blocks $nb --reps 5 > gpurun_out/small/${m}_$nb.json 2>&1 || { echo "$m $nb failed"; tail -5 gpurun_out/small/${m}_$nb.json; exit 1; }
    echo "== $m $nb"; grep GBps gpurun_out/small/${m}_$nb.json
  done
done
