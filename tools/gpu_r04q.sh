# Decoder: short literal runs read before the remap and written after it (parity tests + A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04q
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_periodic.py tests/test_gpu_frames.py > gpurun_out/r04q/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04q/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix,text,copy --reps 7 --so tools/variants/liblz4mi_litov0.so tools/variants/liblz4mi_ab_nolits.so > gpurun_out/r04q/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04q/ab.log; exit $rc
