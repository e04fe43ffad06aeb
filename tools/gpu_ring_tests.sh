set -o pipefail
mkdir -p gpurun_out/r1
export LZ4MI_RING_STATS=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/r1/ring_tests.log 2>&1; echo "ring tests rc=$?"
tail -15 gpurun_out/r1/ring_tests.log
