# Decoder: round-1 literal runs after the match copies (A/B), with outputs cleared between builds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04n
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix,text --reps 7 --so tools/variants/liblz4mi_litlate.so tools/variants/liblz4mi_ab_nolits.so > gpurun_out/r04n/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04n/ab.log; exit $rc
