# Decoder dispatch study: single-pass vs ring vs auto on every generator.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/disp
for m in single ring auto; do
  LZ4MI_DECODER=$m timeout -k 10 300 python tools/microbench.py --gens copy,runs,text,repetitive,per:1000,per:5000,per:40000 --blocks 4096 --reps 3 > gpurun_out/disp/$m.json 2>&1 || { echo "mb $m failed"; tail -20 gpurun_out/disp/$m.json; exit 1; }
  echo "== $m"; grep GBps gpurun_out/disp/$m.json
done
