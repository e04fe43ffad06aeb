# The one GPU runner: every step is time-limited and any failure ends the script (no step runs
# on the GPU after a failed one). STEPS picks and orders the steps; outputs go to gpurun_out/TAG.
#   STEPS="tests bench prof pmc" bash tools/gpu_round.sh TAG
# steps:
#   tests      the GPU suite (PYTEST_ARGS adds selectors, e.g. "-k small")
#   bench      the bench line (BENCH_ARGS adds flags)
#   prof       rocprofv3 --kernel-trace --stats of the bench command (headline + compress only)
#   pmc        FETCH_SIZE / WRITE_SIZE passes of the decode and compress kernels (tools/pmc_traffic.sh)
#   inst       instruction counters of both kernels on the bench workload (one --pmc pass each)
#   small      small-batch latencies (tools/small_latency.py)
#   ab         one-process A/B of the default build against SOS="tools/variants/*.so" (tools/microbench.py,
#              GENS, NBS, WHAT)
#   stress     encoder / small-path stress tools (tools/enc_fuzz.py, tools/small_fuzz.py), SECS seconds each
TAG=${1:-run}
STEPS=${STEPS:-tests bench prof pmc}
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG
for step in $STEPS; do
  case $step in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread $PYTEST_ARGS > $O/pytest.log 2>&1
    rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -12
    [ $rc -eq 0 ] || exit $rc ;;
  bench)
    timeout -k 10 900 python -u bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
    echo "bench ok"; tail -c 4000 $O/bench.json ;;
  prof)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python -u bench.py --steps 5 --warmup 1 --extra 0 --cpu-baseline 0 --napi 0 --frame-blocks 0 > $O/prof_bench.json 2>&1 || { echo rocprof failed; exit 1; }
    echo "rocprof ok" ;;
  pmc)
    timeout -k 10 900 bash tools/pmc_traffic.sh $O/pmc tiles216 > $O/pmc.log 2>&1 || { echo pmc failed; tail -5 $O/pmc.log; exit 1; }
    echo "pmc ok"; tail -12 $O/pmc.log
    timeout -k 10 900 bash tools/pmc_traffic.sh $O/pmc_c tiles216 compress > $O/pmc_c.log 2>&1 || { echo pmc compress failed; tail -5 $O/pmc_c.log; exit 1; }
    echo "pmc compress ok"; tail -12 $O/pmc_c.log ;;
  inst)
    for what in decompress compress; do
      K=lz4mi_decompress_kernel; [ $what = compress ] && K=lz4mi_compress_gts_kernel
      timeout -k 10 300 rocprofv3 --kernel-include-regex $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        -d $O/inst_$what -o pmc --output-format csv -- python tools/microbench.py --what $what --gens tiles216 --blocks 4096 --reps 1 > $O/inst_$what.log 2>&1 || { echo "inst $what failed"; exit 1; }
      echo "inst $what ok"
    done ;;
  small)
    timeout -k 10 300 python -u tools/small_latency.py $SMALL_ARGS > $O/small_latency.log 2>&1 || { echo small failed; tail -5 $O/small_latency.log; exit 1; }
    grep -v amdgpu.ids $O/small_latency.log | tail -20 ;;
  ab)
    for nb in ${NBS:-4096}; do
      timeout -k 10 600 python tools/microbench.py --what ${WHAT:-decompress} --gens ${GENS:-tiles216,random,repetitive} --blocks $nb --reps ${REPS:-3} --so ${SOS:-$(ls tools/variants/*.so 2>/dev/null)} > $O/ab_$nb.log 2>&1 || { echo ab failed; tail -5 $O/ab_$nb.log; exit 1; }
      grep -v amdgpu.ids $O/ab_$nb.log
    done ;;
  stress)
    timeout -k 10 600 python -u tools/enc_fuzz.py --seconds ${SECS:-60} > $O/enc_fuzz.log 2>&1 || { echo enc_fuzz failed; tail -5 $O/enc_fuzz.log; exit 1; }
    tail -3 $O/enc_fuzz.log
    timeout -k 10 600 python -u tools/small_fuzz.py --seconds ${SECS:-60} > $O/small_fuzz.log 2>&1 || { echo small_fuzz failed; tail -5 $O/small_fuzz.log; exit 1; }
    tail -3 $O/small_fuzz.log ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
