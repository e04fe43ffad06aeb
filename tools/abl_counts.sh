# instruction counters of the decode ablation variants (tiles216, 4096 blocks)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ab1 ab2 ab3; do
  timeout -k 10 300 rocprofv3 --kernel-include-regex lz4mi_decompress_kernel --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES -d gpurun_out/abl_$v -o pmc --output-format csv -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 --skip-default --so tools/variants/liblz4mi_$v.so > gpurun_out/abl_$v.log 2>&1 || exit 1
  python tools/pmc_summary.py gpurun_out/abl_$v > gpurun_out/abl_$v.json
done
grep -h "GBps" gpurun_out/abl_*.log
