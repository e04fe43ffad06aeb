# L2 hit/miss and HBM fetch of the batch encoder (tiles216, 4096 x 4 MiB), separate PMC passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ccnt
i=0
for pmc in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex lz4mi_compress_gt_kernel --pmc $pmc -d gpurun_out/ccnt/p$i -o pmc --output-format csv -- python tools/microbench.py --what compress --gens tiles216 --blocks 4096 --reps 1 > gpurun_out/ccnt/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/ccnt/p$i.log; exit 1; }
done
echo ok
