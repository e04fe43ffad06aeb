# Full round (tests, bench, rocprof, PMC traffic), then remap hop limits (A/B) and the output
# phase's instruction split (round 1 only, no piece copies, no remap).
set -o pipefail
cd $GRAFT_REPO_ROOT
STEPS="tests bench prof pmc" bash tools/gpu_round.sh r04s || exit 1
mkdir -p gpurun_out/r04t
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix,text --reps 7 --so tools/variants/liblz4mi_hop2.so tools/variants/liblz4mi_hop4.so > gpurun_out/r04t/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04t/ab.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="abl6 nopipe noremap" bash tools/gpu_phase_valu.sh
