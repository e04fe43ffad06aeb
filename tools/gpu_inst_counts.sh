# Instruction counters of the decode kernel for each named build (tools/variants/), tiles216.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/inst
for v in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-include-regex lz4mi_decompress_kernel --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/inst/$v -o pmc --output-format csv -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 --skip-default --so tools/variants/liblz4mi_$v.so > gpurun_out/inst/$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/inst/$v.log; exit 1; }
done
echo ok
