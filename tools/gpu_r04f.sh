set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04f
timeout -k 10 300 python -u tools/phase_prof.py --gens tiles216 --blocks 4096 > gpurun_out/r04f/phase.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04f/phase.log
bash tools/gpu_r04.sh r04f "tests/test_gpu_parity.py tests/test_gpu_periodic.py tests/test_gpu_frames.py" tiles216,mix,random,text c1 nosplit pb4 def4 || exit 1
timeout -k 10 400 python -u tools/microbench.py --what compress --gens tiles216,mix,text --reps 3 --so tools/variants/liblz4mi_shfl.so tools/variants/liblz4mi_bulk.so > gpurun_out/r04f/cab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r04f/cab.log; exit $rc
