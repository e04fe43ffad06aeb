# Per-phase instruction counts of the decoder: one PMC pass of the 8 SQ counters
# over the 4096 x 4 MiB tiles216 decode for the default build and each ablation build
# (tools/build_variant.sh abl<N> 's/a^//' -DLZ4MI_ABLATE=<N>; N = 3 next table only, 2 parse to the
# walks, 1 no output phase, 6 output round 1 only; abl7/7b/7c: round 1 without its match copies / and
# without the remap / and without the output map, built by sed), then the timings of all of them in one
# process. VARIANTS picks the builds.
#   bash tools/phase_counts.sh OUTDIR            (on the GPU box; tools/phase_counts.py summarises)
set -o pipefail
O=${1:-gpurun_out/phase}
mkdir -p $O
export TMPDIR=/tmp
CNT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for v in ${VARIANTS:-default abl3 abl2 abl1 abl6}; do
  extra=""; [ $v = default ] || extra="--skip-default --so tools/variants/liblz4mi_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-include-regex lz4mi_decompress_kernel --pmc $CNT -d $O/$v -o pmc --output-format csv \
    -- python tools/microbench.py --what decompress --gens tiles216 --blocks 4096 --reps 1 $extra > $O/$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/$v.log; exit 1; }
  echo "pmc $v ok"
done
timeout -k 10 600 python tools/microbench.py --what decompress --gens tiles216 --blocks 4096 --reps 5 \
  --so $(for v in ${VARIANTS:-default abl3 abl2 abl1 abl6}; do [ $v = default ] || echo tools/variants/liblz4mi_$v.so; done) > $O/times.log 2>&1 || { echo "times failed"; tail -5 $O/times.log; exit 1; }
grep -v amdgpu.ids $O/times.log
