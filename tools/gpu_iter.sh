# One iteration: GPU tests, ring-decoder phase profile, bench (auto dispatch) vs single-pass only.
set -o pipefail
O=gpurun_out/${1:-it}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for g in ${GENS:-}; do
LZ4MI_DECODER=ring LZ4MI_RING_STATS=1 timeout -k 10 200 python tools/ring_prof.py --so tools/variants/liblz4mi_ringprof.so --gen $g > $O/prof_$g.txt 2>&1 || { echo fail; tail -20 $O/prof_$g.txt; exit 1; }
grep -v amdgpu.ids $O/prof_$g.txt
done
summ() { python - $1 <<'PY'
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[1], "tiles216 decode GB/s", d["value"], "ms", d["ms_per_step"], {k:v["decompress_GBps"] for k,v in d.get("variants",{}).items()})
PY
}
timeout -k 10 300 python bench.py --steps 10 --extra ${EXTRA:-1} --cpu-baseline 0 --frame-steps 0 --compress-steps 1 > $O/auto.json 2> $O/auto.err || { echo "bench failed"; tail -20 $O/auto.err; exit 1; }
summ $O/auto.json
if [ -n "${SINGLE:-}" ]; then
LZ4MI_DECODER=single timeout -k 10 300 python bench.py --steps 10 --extra ${EXTRA:-1} --cpu-baseline 0 --frame-steps 0 --compress-steps 1 > $O/single.json 2> $O/single.err || { echo "bench failed"; tail -20 $O/single.err; exit 1; }
summ $O/single.json
fi
