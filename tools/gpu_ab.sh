# A/B of the decoders: the ring (two-pass) default vs the single-pass kernel, plus the GPU tests.
set -o pipefail
O=gpurun_out/${1:-ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --steps 10 --extra ${EXTRA:-1} --cpu-baseline 0 --frame-steps 0 --compress-steps 1 > $O/ring.json 2> $O/ring.err || { echo "ring bench failed"; tail -20 $O/ring.err; exit 1; }
cat $O/ring.json
LZ4MI_DECODER=single timeout -k 10 300 python bench.py --steps 10 --extra 0 --cpu-baseline 0 --frame-steps 0 --compress-steps 1 > $O/single.json 2> $O/single.err || { echo "single bench failed"; tail -20 $O/single.err; exit 1; }
cat $O/single.json
