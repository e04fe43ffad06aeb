# Encoder: hit-batch probe count without a division (A/B + parity), then the decoder's
# per-phase instruction counts.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04r
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r04r/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04r/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216,mix,text --reps 3 --so tools/variants/liblz4mi_kdiv.so tools/variants/liblz4mi_off64.so tools/variants/liblz4mi_noslot.so > gpurun_out/r04r/cab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04r/cab.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_phase_valu.sh
