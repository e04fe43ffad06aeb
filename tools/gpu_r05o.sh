# round-5 encoder read accounting: FETCH_SIZE of a build that repeats every table read from the
# never-written upper half of the block's table slot (the difference from the default build's
# 243 GB = the table reads' fetch), and its time beside the default (traffic sensitivity)
cd $GRAFT_REPO_ROOT && T=${1:-r05o} && mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216,mix --reps 3 --so tools/variants/liblz4mi_shadowrd.so tools/variants/liblz4mi_shadow.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/shadow_time.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-include-regex lz4mi_compress_gts_kernel --pmc FETCH_SIZE -d gpurun_out/$T/pmc_shadowrd/FETCH_SIZE -o pmc \
  --output-format csv -- python tools/microbench.py --what compress --gens tiles216 --blocks 4096 --reps 1 --so tools/variants/liblz4mi_shadowrd.so --skip-default > gpurun_out/$T/pmc_shadowrd.log 2>&1 || { echo "pass failed"; exit 1; }
echo pass ok
