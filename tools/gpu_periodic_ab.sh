# LDS periodic-run path: GPU tests, then A/B against the history re-read variant
# (tools/variants/liblz4mi_noper.so) with the single-pass kernel, and the ring decoder.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/per
timeout -k 10 400 python -u -m pytest tests/test_gpu_periodic.py tests/test_gpu_parity.py tests/test_gpu_ring.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/per/pytest.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/per/pytest.log; exit 1; }
tail -3 gpurun_out/per/pytest.log
G=${GENS:-repetitive,per:1000,per:5000,per:40000,per:65000,tiles216,random}
LZ4MI_DECODER=single timeout -k 10 400 python tools/microbench.py --gens $G --blocks 4096 --reps 5 --so tools/variants/liblz4mi_noper.so > gpurun_out/per/single.json 2>&1 || { echo "mb single failed"; tail -20 gpurun_out/per/single.json; exit 1; }
grep GBps gpurun_out/per/single.json
LZ4MI_DECODER=ring timeout -k 10 300 python tools/microbench.py --gens per:5000,per:40000,per:65000 --blocks 4096 --reps 3 > gpurun_out/per/ring.json 2>&1 || { echo "mb ring failed"; tail -20 gpurun_out/per/ring.json; exit 1; }
grep GBps gpurun_out/per/ring.json
