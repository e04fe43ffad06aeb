# round-5 small-batch decode latency: pointer-jumping path vs the batch kernel (1..16 blocks),
# and a kernel trace of the small path (parse / expand / jump rounds / gather)
cd $GRAFT_REPO_ROOT && T=${1:-r05s} && mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/small_latency.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/small.log || exit 1
LZ4MI_SMALL_BLOCKS=0 timeout -k 10 300 python -u tools/small_latency.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/batch.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python -u tools/small_latency.py --gens tiles216 --counts 1 --reps 3 > gpurun_out/$T/prof.log 2>&1 || { echo prof failed; exit 1; }
echo prof ok
