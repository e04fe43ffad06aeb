# GPU tests, then A/B microbench of the default build against tools/variants/*.so
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1; tail -4 gpurun_out/t.log
for nb in ${NBS:-4096}; do
timeout -k 10 400 python tools/microbench.py --gens ${GENS:-tiles216,random,repetitive} --blocks $nb --reps 3 --so ${SOS:-$(ls tools/variants/*.so 2>/dev/null)} > gpurun_out/mb.log 2>&1; grep -v amdgpu.ids gpurun_out/mb.log
done
