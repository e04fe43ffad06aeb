# Decoder: long literal copies throttled (s_sleep per 4 KiB step) on the skewed mix (A/B).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ll
timeout -k 10 300 python -u tools/microbench.py --gens mix,random,tiles216 --reps 7 --so tools/variants/liblz4mi_llsleep.so tools/variants/liblz4mi_llsleep16.so > gpurun_out/ll/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ll/ab.log; exit $rc
