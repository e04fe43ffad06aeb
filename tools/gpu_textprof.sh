# Phase profile of the single-pass decoder on text/runs/copy vs tiles216, and the
# far-copy generator under each decoder.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tp
LZ4MI_DECODER=single timeout -k 10 400 python tools/phase_prof.py --gens tiles216,text,runs,copy --blocks 4096 > gpurun_out/tp/phase.log 2>&1 || { echo "phase failed"; tail -20 gpurun_out/tp/phase.log; exit 1; }
cat gpurun_out/tp/phase.log
for m in single ring; do
LZ4MI_DECODER=$m timeout -k 10 300 python tools/microbench.py --gens far --blocks 4096 --reps 3 > gpurun_out/tp/far_$m.json 2>&1 || { echo "far failed"; tail -20 gpurun_out/tp/far_$m.json; exit 1; }
echo $m; grep GBps gpurun_out/tp/far_$m.json
done
