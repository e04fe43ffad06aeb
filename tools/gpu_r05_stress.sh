# randomized decode stress over every path: small batches and the batch kernel, spec and
# reference mode, encoder output with corruptions and random valid streams (50 s each)
set -o pipefail
cd $GRAFT_REPO_ROOT && T=${1:-r05_stress} && mkdir -p gpurun_out/$T
run() { timeout -k 10 150 python -u tools/small_fuzz.py --seconds 50 --dump gpurun_out/$T/d_$1 "${@:2}" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/$T/stress.log; }
run a --seed 31 --min-blocks 97 --max-blocks 200 || exit 1
run b --seed 32 --js-exact || exit 1
run c --seed 33 --js-exact --min-blocks 97 --max-blocks 160 || exit 1
run d --seed 34 --random-streams || exit 1
run e --seed 35 --random-streams --min-blocks 97 --max-blocks 200 || exit 1
