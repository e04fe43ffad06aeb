cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r02a.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_r02a.log
if [ $rc -le 1 ]; then
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --extra 0 > gpurun_out/bench_r02a.log 2>&1
  echo "bench rc=$?"
  tail -c 3000 gpurun_out/bench_r02a.log
fi
