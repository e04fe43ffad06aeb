# Speculative hit-chain encoder: parity tests, then A/B against the one-probe-per-round-trip kernel.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03b/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r03b/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/compress_ab.py --gens tiles216,random,text,copy,runs,repetitive --blocks 4096 --enc gt > gpurun_out/r03b/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03b/ab.log; exit $rc
