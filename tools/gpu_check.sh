# Full GPU test suite, then an optional A/B script.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/chk
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/chk/pytest.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/chk/pytest.log; exit 1; }
tail -3 gpurun_out/chk/pytest.log
if [ -n "$1" ]; then s=$1; shift; bash $s "$@"; fi
