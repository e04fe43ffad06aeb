# GPU parity tests + encoder/chain timings of the current build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$1/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/$1/pytest.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216,random --reps 3 > gpurun_out/$1/comp.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$1/comp.log
timeout -k 10 300 python -u tools/chain_time.py tiles216,random > gpurun_out/$1/chain.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/$1/chain.log
