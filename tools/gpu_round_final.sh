# End-of-round GPU pass: parity tests, the PMC HBM-traffic passes of the decode kernel
# (copied to profiles/pmc_traffic.json so the bench line carries them), the bench line,
# and rocprofv3 kernel stats of the bench command. Each step is time-limited; any
# failure ends the script.
#   bash tools/gpu_round_final.sh TAG
TAG=${1:-final}
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/$TAG/pytest.log | tail -3
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 bash tools/pmc_traffic.sh gpurun_out/$TAG/pmc tiles216 > gpurun_out/$TAG/pmc.log 2>&1 || { echo pmc failed; tail -5 gpurun_out/$TAG/pmc.log; exit 1; }
cp gpurun_out/$TAG/pmc/pmc_traffic.json profiles/pmc_traffic.json
echo "pmc ok"; tail -12 gpurun_out/$TAG/pmc.log
timeout -k 10 600 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo bench failed; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
echo "bench ok"; tail -c 1500 gpurun_out/$TAG/bench.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python -u bench.py --steps 5 --warmup 1 --extra 0 --cpu-baseline 0 --napi 0 --frame-steps 0 > gpurun_out/$TAG/prof_bench.json 2>&1 || { echo rocprof failed; exit 1; }
echo "rocprof ok"
