# round-5 small-batch decode: phase-1 re-parse tests (natural and forced), then the whole suite
cd $GRAFT_REPO_ROOT && T=${1:-r05w} && mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/small.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tests.log || exit 1
