# LDS hand-offs by compiler fence (LZ4MI_WSYNC) vs __syncthreads: timing and exact output on every generator
cd $GRAFT_REPO_ROOT && T=${1:-r05h} && mkdir -p gpurun_out/$T
timeout -k 10 900 python -u tools/microbench.py --gens tiles216,mix,random,repetitive,copy,text,per:1000,far --reps 5 --so tools/variants/liblz4mi_wsync.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/ab.log
