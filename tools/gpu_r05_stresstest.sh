# the seeded stress tests, then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT && T=${1:-r05_stresstest} && mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_stress.py -m gpu -x -v --timeout 200 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/stress_tests.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tests.log || exit 1
