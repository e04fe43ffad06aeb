# Decoder ablations (timing only except noremap, which is a valid build): literal runs, piece loads, remap.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04m
timeout -k 10 300 python -u tools/microbench.py --gens tiles216 --reps 7 --so tools/variants/liblz4mi_ab_nolits.so tools/variants/liblz4mi_ab_noload.so tools/variants/liblz4mi_ab_noremap.so > gpurun_out/r04m/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04m/ab.log; exit $rc
