# the window-edge test (fixed reference-mode expectation) and the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT && T=${1:-r05_edge2} && mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tests.log || exit 1
