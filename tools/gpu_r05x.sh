# round-5 final pass: small-batch tests and latency (per-thread done bytes in the jump rounds),
# then tools/gpu_round.sh (GPU suite, bench line, rocprof of the bench, PMC traffic passes)
cd $GRAFT_REPO_ROOT && T=${1:-r05x} && mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/small.log || exit 1
timeout -k 10 300 python -u tools/small_latency.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/latency.log || exit 1
bash tools/gpu_round.sh $T
