# small-batch decode: ratio >= 32 blocks by one wave, threshold 96 -- the GPU suite, latency
cd $GRAFT_REPO_ROOT && T=${1:-r06d} && mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tests.log || exit 1
timeout -k 10 300 python -u tools/small_latency.py --counts 1,4,16,64,96 --reps 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/latency.log || exit 1
