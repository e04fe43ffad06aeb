cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_js_shim.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r03e/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/chain_ab.py tiles216,text,random,copy > gpurun_out/r03e/chain.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03e/chain.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/compress_ab.py --gens tiles216,random,repetitive --blocks 4096 --enc gt > gpurun_out/r03e/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03e/ab.log; exit $rc
