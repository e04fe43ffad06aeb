# Decoder: remap following earlier rows' mappings in one step (parity tests + A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04u
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_periodic.py tests/test_gpu_frames.py > gpurun_out/r04u/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04u/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix,text,copy --reps 7 --so tools/variants/liblz4mi_memo0.so > gpurun_out/r04u/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04u/ab.log; exit $rc
