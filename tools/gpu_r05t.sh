# round-5 small-batch decode (segment-parallel parse, verify kernel, done-flag jump rounds): its tests, the whole GPU suite, the small-batch
# latency (path on / off), and the batch kernel against the previous commit's (DecArgs grew)
cd $GRAFT_REPO_ROOT && T=${1:-r05t} && mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/small.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tests.log || exit 1
timeout -k 10 300 python -u tools/small_latency.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/latency.log || exit 1
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix,random --reps 5 --so tools/variants/liblz4mi_prev.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/batch_ab.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python -u tools/small_latency.py --gens tiles216 --counts 1,16 --reps 3 > gpurun_out/$T/prof.log 2>&1 || { echo prof failed; exit 1; }
echo prof ok
