# small-batch decode, adaptive segments (<= 256 of ~8 KiB) with phase 2 (the first wrong segment
# (all of them at once, twice), then the check again): the GPU suite, latency, per-dispatch kernel times
cd $GRAFT_REPO_ROOT && T=${1:-r05s2_k} && mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/small.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tests.log || exit 1
timeout -k 10 300 python -u tools/small_latency.py --counts 1,4,16,64,96 --reps 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/latency.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run -- python3 tools/small_latency.py --counts 1,64 --reps 2 --gens text > gpurun_out/$T/prof.log 2>&1 || exit 1
