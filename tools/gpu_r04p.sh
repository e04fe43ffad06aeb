# Decoder diagnostic: literal stores to an LDS sink instead of the output (timing only).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04p
timeout -k 10 300 python -u tools/microbench.py --gens tiles216 --reps 7 --so tools/variants/liblz4mi_litsink.so tools/variants/liblz4mi_litsink2.so tools/variants/liblz4mi_ab_nolits.so > gpurun_out/r04p/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04p/ab.log; exit $rc
