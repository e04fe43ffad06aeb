# Encoder: lane gathers as raw ds_bpermute (parity + A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04y
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_frames.py > gpurun_out/r04y/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04y/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216,mix,random --reps 3 --so tools/variants/liblz4mi_shfl.so > gpurun_out/r04y/cab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04y/cab.log; exit $rc
