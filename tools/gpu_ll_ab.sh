# Decoder: long literal runs copied with nontemporal loads/stores (parity tests + A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ll
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_frames.py > gpurun_out/ll/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/ll/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --gens mix,random,tiles216 --reps 7 --so tools/variants/liblz4mi_nt0.so > gpurun_out/ll/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ll/ab.log; exit $rc
