# Decoder: two-pass remap (parity tests + A/B: one pass, first pass of 1 / 3 hops).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/remap2
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_periodic.py tests/test_gpu_frames.py > gpurun_out/remap2/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/remap2/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix,text,copy --reps 7 --so tools/variants/liblz4mi_onepass.so tools/variants/liblz4mi_pass1.so tools/variants/liblz4mi_pass3.so > gpurun_out/remap2/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/remap2/ab.log; exit $rc
