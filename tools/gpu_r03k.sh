cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03k
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03k/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r03k/pytest.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/microbench.py --gens tiles216,mix,random --reps 7 --so tools/variants/liblz4mi_base.so tools/variants/liblz4mi_wshr.so > gpurun_out/r03k/micro.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03k/micro.log
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216,random,repetitive --reps 3 --so tools/variants/liblz4mi_base.so > gpurun_out/r03k/comp.log 2>&1
grep -v amdgpu.ids gpurun_out/r03k/comp.log
