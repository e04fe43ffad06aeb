# fuzz over both decode paths (small-batch and batch kernel), then the whole GPU suite
cd $GRAFT_REPO_ROOT && T=${1:-r05s2_l} && mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_parity.py -k "fuzz" -m gpu -x -v --timeout 120 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/fuzz.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tests.log || exit 1
