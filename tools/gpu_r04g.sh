# Round-4 GPU batch: decoder phase profile, parity tests, decode and encode A/B against the
# variant builds, then every other GPU test and the full bench line (one box, one call).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04g
bash tools/gpu_r04f.sh || exit 1
cp -r gpurun_out/r04f/. gpurun_out/r04g/
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  --ignore=tests/test_gpu_parity.py --ignore=tests/test_gpu_periodic.py --ignore=tests/test_gpu_frames.py \
  > gpurun_out/r04g/pytest_rest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04g/pytest_rest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r04g/bench.json 2> gpurun_out/r04g/bench.err || { echo bench failed; tail -20 gpurun_out/r04g/bench.err; exit 1; }
echo bench ok; tail -c 4000 gpurun_out/r04g/bench.json
