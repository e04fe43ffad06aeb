# GPU check: the given pytest selection (default: all GPU tests; "none" skips), then the
# decode microbench on the given generators (MB_ARGS: extra microbench args, e.g. --so ...).
# Each step time-limited; a failure ends it.
#   bash tools/gpu_check.sh TAG [pytest-args|none] [gens]
TAG=${1:-chk}; SEL=${2:-tests}; GENS=${3:-tiles216,random,repetitive,mix}
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG
if [ "$SEL" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $SEL -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/$TAG/pytest.log | tail -8
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u tools/microbench.py --gens $GENS --reps 7 $MB_ARGS > gpurun_out/$TAG/micro.log 2>&1
rc=$?; grep -v Warn gpurun_out/$TAG/micro.log | tail -16; exit $rc
