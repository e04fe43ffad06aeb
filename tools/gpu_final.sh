# Final pass of a round: tools/gpu_round.sh (GPU suite, bench line, rocprof of the bench command,
# PMC traffic passes), then the instruction counters of the decode and compress kernels on the
# bench workload (one --pmc pass each, 8 SQ counters) and the small-batch latencies
cd $GRAFT_REPO_ROOT && T=${1:-final} && mkdir -p gpurun_out/$T
bash tools/gpu_round.sh $T || exit 1
export TMPDIR=/tmp
for what in decompress compress; do
  K=lz4mi_decompress_kernel; [ $what = compress ] && K=lz4mi_compress_gts_kernel
  timeout -k 10 300 rocprofv3 --kernel-include-regex $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d gpurun_out/$T/inst_$what -o pmc --output-format csv -- python tools/microbench.py --what $what --gens tiles216 --blocks 4096 --reps 1 > gpurun_out/$T/inst_$what.log 2>&1 || { echo "inst $what failed"; exit 1; }
  echo "inst $what ok"
done
timeout -k 10 300 python -u tools/small_latency.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/small_latency.log || exit 1
