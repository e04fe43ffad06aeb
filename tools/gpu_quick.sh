# quick GPU iteration: the given pytest selection, then optional extra command
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $1 -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/quick.log | tail -30
[ $rc -le 1 ] || exit $rc
if [ -n "$2" ]; then timeout -k 10 600 bash -c "$2" > gpurun_out/quick_extra.log 2>&1; echo "extra rc=$?"; tail -c 2500 gpurun_out/quick_extra.log; fi
