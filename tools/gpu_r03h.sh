cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03h
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03h/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r03h/pytest.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/microbench.py --gens tiles216,mix,random,repetitive,text,copy --reps 5 --so tools/variants/liblz4mi_dec_r02.so > gpurun_out/r03h/micro.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03h/micro.log
timeout -k 10 300 python -u tools/chain_time.py tiles216,text,random > gpurun_out/r03h/chain.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03h/chain.log
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216,random --reps 3 --so tools/variants/liblz4mi_gt16.so > gpurun_out/r03h/comp.log 2>&1
grep -v amdgpu.ids gpurun_out/r03h/comp.log
