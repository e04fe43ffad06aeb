# round-5 encoder A/B: hit-batch window loads without per-lane bounds branches (winu), and the
# probe bytes' LDS read without its exec-mask branch too (winu2); byte-identical check + time
cd $GRAFT_REPO_ROOT && T=${1:-r05z} && mkdir -p gpurun_out/$T
timeout -k 10 500 python -u tools/microbench.py --what compress --gens tiles216,mix,random --reps 5 --so tools/variants/liblz4mi_winu.so tools/variants/liblz4mi_winu2.so tools/variants/liblz4mi_winu3.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/cab.log
