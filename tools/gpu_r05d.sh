# round-5: block dispatch order + adaptive long-literal pacing (defaults) vs their ablations,
# timelines of the default and the round-4 behaviour, then the GPU tests
cd $GRAFT_REPO_ROOT && T=${1:-r05d} && mkdir -p gpurun_out/$T
so=""; for v in noord ord2 base4 ad96; do so="$so tools/variants/liblz4mi_$v.so"; done
timeout -k 10 600 python -u tools/microbench.py --gens tiles216,mix,mixc,random,repetitive --reps 7 --so $so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/ab.log || exit 1
timeout -k 10 300 python -u tools/timeline.py --so tools/variants/liblz4mi_tl.so --gens tiles216,mix,mixc --out gpurun_out/$T/tl 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/timeline_tl.log || exit 1
timeout -k 10 300 python -u tools/timeline.py --so tools/variants/liblz4mi_base4tl.so --gens tiles216 --out gpurun_out/$T/base 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/timeline_base.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/$T/pytest.log | tail -8; exit $rc
