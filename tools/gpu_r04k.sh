# Round-4 A/B: remap bucket size and piece batch (decode); emission share of the encoder
# (timing-only build without emission: its output is not valid).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04k
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix --reps 7 --so tools/variants/liblz4mi_msh5.so tools/variants/liblz4mi_pb12.so > gpurun_out/r04k/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04k/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216,mix --reps 3 --so tools/variants/liblz4mi_noemit.so > gpurun_out/r04k/cab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04k/cab.log; exit $rc
