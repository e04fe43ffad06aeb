# VALU / SALU / LDS instructions of the decoder by phase: the ablation builds (1 = no output,
# 2 = parse to the walks, 3 = next-token table only) against the default, tiles216 4096 x 4 MiB.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pv
for v in ${VARIANTS:-abl1 abl2 abl3}; do
  timeout -s KILL 120 rocprofv3 --kernel-include-regex lz4mi_decompress_kernel --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    -d gpurun_out/pv/$v -o pmc --output-format csv -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 \
    --so tools/variants/liblz4mi_$v.so > gpurun_out/pv/$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/pv/$v.log; exit 1; }
  echo "$v: $(python tools/phase_valu.py gpurun_out/pv/$v)"
done
