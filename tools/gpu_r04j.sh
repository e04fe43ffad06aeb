# Decoder phase profile with the round-1 split, then the PMC counter passes of both kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04j
timeout -k 10 300 python -u tools/phase_prof.py --gens tiles216 --blocks 1024,4096 > gpurun_out/r04j/phase.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04j/phase.log
bash tools/gpu_counters.sh
