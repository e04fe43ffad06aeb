# round-5: wave-priority rotation (decoder, encoder) vs the defaults; encoder per-block timeline
cd $GRAFT_REPO_ROOT && T=${1:-r05e} && mkdir -p gpurun_out/$T
timeout -k 10 600 python -u tools/microbench.py --gens tiles216,mix,random,repetitive --reps 7 --so tools/variants/liblz4mi_rot1.so tools/variants/liblz4mi_rot2.so tools/variants/liblz4mi_base4.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/ab.log || exit 1
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216,mix --reps 3 --so tools/variants/liblz4mi_cpr2.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/cab.log || exit 1
timeout -k 10 300 python -u tools/timeline.py --what compress --so tools/variants/liblz4mi_ctl.so --gens tiles216 --out gpurun_out/$T/ctl 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/ctimeline.log || exit 1
timeout -k 10 300 python -u tools/timeline.py --so tools/variants/liblz4mi_rot2tl.so --gens tiles216 --out gpurun_out/$T/rot2 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/timeline_rot2.log || exit 1
