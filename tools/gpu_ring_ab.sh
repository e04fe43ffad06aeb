# Ring decoder (opt-in): its GPU tests, then A/B of two builds with every block through it.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ringab
timeout -k 10 400 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_periodic.py tests/test_gpu_frames.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/ringab/pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ringab/pytest.log; exit 1; }
tail -1 gpurun_out/ringab/pytest.log
LZ4MI_DECODER=ring timeout -k 10 400 python tools/microbench.py --gens tiles216,repetitive,per:40000,random --blocks 4096 --reps 3 --skip-default --so tools/variants/liblz4mi_$1.so tools/variants/liblz4mi_$2.so > gpurun_out/ringab/ab.json 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ringab/ab.json; exit 1; }
grep GBps gpurun_out/ringab/ab.json
