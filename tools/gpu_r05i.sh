# the `far` round-trip failure: encoder vs decoder, and which decoder change
cd $GRAFT_REPO_ROOT && T=${1:-r05i} && mkdir -p gpurun_out/$T
timeout -k 10 600 python -u tools/far_check.py --n 64 --so tools/variants/liblz4mi_noord.so tools/variants/liblz4mi_noad.so tools/variants/liblz4mi_base4.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/far.log
