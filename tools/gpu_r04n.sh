# Decoder: round-1 literal runs after the match copies (A/B, outputs cleared between builds);
# encoder: epoch-code inserts as ds_mskor (parity tests + A/B against LDS atomic AND + OR).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04n
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r04n/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r04n/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix,text --reps 7 --so tools/variants/liblz4mi_litlate.so tools/variants/liblz4mi_ab_nolits.so > gpurun_out/r04n/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04n/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216,mix --reps 3 --so tools/variants/liblz4mi_nomskor.so > gpurun_out/r04n/cab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04n/cab.log; exit $rc
