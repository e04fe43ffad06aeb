# small-batch decode: jump rounds and chase in a strided (coalesced) layout -- tests, latency
cd $GRAFT_REPO_ROOT && T=${1:-r06b} && mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/small.log || exit 1
timeout -k 10 300 python -u tools/small_latency.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/latency.log || exit 1
LZ4MI_SMALL_BLOCKS=64 timeout -k 10 300 python -u tools/small_latency.py --gens tiles216,text --counts 32,48,64 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/latency_big.log || exit 1
