# round-5 decoder A/B: long-literal depth/pacing and wave-priority modes
# (age arbitration), timelines of the best candidates, then the GPU tests
cd $GRAFT_REPO_ROOT && T=${1:-r05c} && mkdir -p gpurun_out/$T
so=""; for v in d1 d4s127 ad64 ad127 pr1 pr2 pr3 p32 p32pr1; do so="$so tools/variants/liblz4mi_$v.so"; done
timeout -k 10 600 python -u tools/microbench.py --gens tiles216,mix,mixc,random,repetitive --reps 7 --so $so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/ab.log || exit 1
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216,mix --reps 3 --so tools/variants/liblz4mi_cpr1.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/cab.log || exit 1
timeout -k 10 300 python -u tools/timeline.py --so tools/variants/liblz4mi_pr1tl.so --gens tiles216,mix --out gpurun_out/$T/pr1 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/timeline_pr1.log || exit 1
timeout -k 10 300 python -u tools/timeline.py --so tools/variants/liblz4mi_ad127tl.so --gens mixc --out gpurun_out/$T/ad127 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/timeline_ad127.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/$T/pytest.log | tail -8; exit $rc
