# Round-4: encoder emission by sequence lanes (parity tests + A/B against the old emission),
# remap map granule 64 B vs 32 B (decode A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04l
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_frames.py > gpurun_out/r04l/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04l/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216,mix,text --reps 3 --so tools/variants/liblz4mi_emit0.so > gpurun_out/r04l/cab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04l/cab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix,text --reps 7 --so tools/variants/liblz4mi_msh6.so > gpurun_out/r04l/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04l/ab.log; exit $rc
