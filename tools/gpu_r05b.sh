# round-5 experiment set: decoder A/B (hygiene build vs round-4 base vs sc1 literal stores),
# the mix timeline, and the decode latency curve (1 .. 4096 blocks)
cd $GRAFT_REPO_ROOT && T=${1:-r05b} && mkdir -p gpurun_out/$T
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix,random,repetitive --reps 7 \
  --so tools/variants/liblz4mi_base.so tools/variants/liblz4mi_litsc1.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/ab.log || exit 1
timeout -k 10 300 python -u tools/timeline.py --so tools/variants/liblz4mi_tl.so --gens mix,mixc,tiles216 --out gpurun_out/$T 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/timeline.log || exit 1
for nb in 1 16 256 2048 4096; do
  timeout -k 10 120 python -u tools/microbench.py --gens tiles216 --blocks $nb --reps 7 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/$T/latency.log || exit 1
done
