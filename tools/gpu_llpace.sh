# long-literal copy depth / pacing variants on the mixes, then the GPU tests
cd $GRAFT_REPO_ROOT && T=${1:-r05c} && mkdir -p gpurun_out/$T
so=""; for v in d1 d4s64 d4s127 d2s127 ad64 ad127; do so="$so tools/variants/liblz4mi_$v.so"; done
timeout -k 10 500 python -u tools/microbench.py --gens mix,mixc,random,tiles216 --reps 7 --so $so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/ab.log || exit 1
timeout -k 10 300 python -u tools/timeline.py --so tools/variants/liblz4mi_ad127tl.so --gens mix,mixc --out gpurun_out/$T 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/timeline.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/$T/pytest.log | tail -8; exit $rc
