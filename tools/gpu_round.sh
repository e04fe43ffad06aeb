# Round GPU pass: parity tests, the bench line, rocprofv3 kernel stats of the bench
# command and the PMC HBM-traffic passes of the decode kernel. Each step is time-limited;
# any failure ends the script. STEPS selects a subset (default: all).
#   STEPS="tests bench prof pmc" bash tools/gpu_round.sh TAG
TAG=${1:-r03}
STEPS=${STEPS:-tests bench prof pmc}
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/$TAG/pytest.log | tail -8
  [ $rc -le 1 ] || exit $rc
fi
if has bench; then
  timeout -k 10 900 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo bench failed; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
  echo "bench ok"; tail -c 3000 gpurun_out/$TAG/bench.json
fi
export TMPDIR=/tmp
if has prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python -u bench.py --steps 5 --warmup 1 --extra 0 --cpu-baseline 0 --napi 0 --frame-blocks 0 > gpurun_out/$TAG/prof_bench.json 2>&1 || { echo rocprof failed; exit 1; }
  echo "rocprof ok"
fi
if has pmc; then
  timeout -k 10 900 bash tools/pmc_traffic.sh gpurun_out/$TAG/pmc tiles216 > gpurun_out/$TAG/pmc.log 2>&1 || { echo pmc failed; tail -5 gpurun_out/$TAG/pmc.log; exit 1; }
  echo "pmc ok"; tail -12 gpurun_out/$TAG/pmc.log
  timeout -k 10 900 bash tools/pmc_traffic.sh gpurun_out/$TAG/pmc_c tiles216 compress > gpurun_out/$TAG/pmc_c.log 2>&1 || { echo pmc compress failed; tail -5 gpurun_out/$TAG/pmc_c.log; exit 1; }
  echo "pmc compress ok"; tail -12 gpurun_out/$TAG/pmc_c.log
fi
