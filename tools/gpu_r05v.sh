# round-5 small-batch decode: tests, the whole GPU suite, latency 1..16 (default threshold),
# 16..64 blocks with the threshold raised vs the batch kernel (crossover), kernel trace
cd $GRAFT_REPO_ROOT && T=${1:-r05v} && mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/small.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tests.log || exit 1
timeout -k 10 300 python -u tools/small_latency.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/latency.log || exit 1
LZ4MI_SMALL_BLOCKS=64 timeout -k 10 300 python -u tools/small_latency.py --gens tiles216,text --counts 16,24,32,48,64 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/latency_big_small.log || exit 1
LZ4MI_SMALL_BLOCKS=0 timeout -k 10 300 python -u tools/small_latency.py --gens tiles216,text --counts 16,24,32,48,64 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/latency_big_batch.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python -u tools/small_latency.py --gens tiles216,text --counts 1,16 --reps 3 > gpurun_out/$T/prof.log 2>&1 || { echo prof failed; exit 1; }
echo prof ok
