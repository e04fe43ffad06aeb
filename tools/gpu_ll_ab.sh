# Decoder: nontemporal streams — long literal runs (default on; nt0 = off), the staged compressed
# stream (stagent), long periodic runs' stores (pernt): parity tests + A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ll2
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_periodic.py tests/test_gpu_frames.py > gpurun_out/ll2/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/ll2/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/microbench.py --gens tiles216,mix,random,repetitive --reps 7 --so tools/variants/liblz4mi_nt0.so tools/variants/liblz4mi_stagent.so tools/variants/liblz4mi_pernt.so > gpurun_out/ll2/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ll2/ab.log; exit $rc
