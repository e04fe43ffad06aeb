# round-5 encoder fix (ring_copy: literal runs of 2034..2048 bytes wrapped the batch encoder's
# 2 KiB output ring): the `far` blocks vs the oracle, then the whole GPU suite
cd $GRAFT_REPO_ROOT && T=${1:-r05k} && mkdir -p gpurun_out/$T
timeout -k 10 300 python -u tools/far_check.py --n 64 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/far.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tests.log
