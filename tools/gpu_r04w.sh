# Compiler scheduling options for both kernels (A/B against the default build).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04w
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix --reps 7 --so tools/variants/liblz4mi_fbias0.so tools/variants/liblz4mi_fbias100.so tools/variants/liblz4mi_ftrk.so > gpurun_out/r04w/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04w/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216 --reps 3 --so tools/variants/liblz4mi_fbias0.so tools/variants/liblz4mi_fbias100.so tools/variants/liblz4mi_ftrk.so > gpurun_out/r04w/cab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04w/cab.log; exit $rc
