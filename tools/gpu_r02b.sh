cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dbg_bcs.py > gpurun_out/dbg_bcs.log 2>&1; echo "dbg rc=$?"; cat gpurun_out/dbg_bcs.log | tail -40
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r02b.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASS|FAIL|Error" gpurun_out/pytest_r02b.log | tail -40
