cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03l
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_js_shim.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03l/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r03l/pytest.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/chain_time.py tiles216,text,random > gpurun_out/r03l/chain.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03l/chain.log
timeout -k 10 300 python -u tools/chain_prof.py tiles216,text > gpurun_out/r03l/cprof.log 2>&1
grep -v amdgpu.ids gpurun_out/r03l/cprof.log
