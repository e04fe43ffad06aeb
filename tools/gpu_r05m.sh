# round-5 encoder A/B: probes per hit batch (static 4 / 6, adaptive J + 2 / 2 (J + 1)) against
# the default 8 -- speculative probes past the batch's end fetch table and window lines for nothing
cd $GRAFT_REPO_ROOT && T=${1:-r05m} && mkdir -p gpurun_out/$T
so=""; for v in k4 k6 ka1 ka2; do so="$so tools/variants/liblz4mi_$v.so"; done
timeout -k 10 500 python -u tools/microbench.py --what compress --gens tiles216,mix,copy,text --reps 3 --so $so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/cab.log
