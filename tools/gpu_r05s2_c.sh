# small-batch decode crossover with the coalesced rounds: 64..256 blocks, small path vs batch kernel
cd $GRAFT_REPO_ROOT && T=${1:-r06c} && mkdir -p gpurun_out/$T
LZ4MI_SMALL_BLOCKS=256 timeout -k 10 400 python -u tools/small_latency.py --gens tiles216,text,repetitive --counts 64,96,128,192,256 --reps 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/small.log || exit 1
LZ4MI_SMALL_BLOCKS=0 timeout -k 10 400 python -u tools/small_latency.py --gens tiles216,text,repetitive --counts 64,128,256 --reps 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/batch.log || exit 1
