# Decoder wave priorities by phase (A/B): walks 2; next table 1 + walks 2; output 2.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/prio
timeout -k 10 300 python -u tools/microbench.py --gens tiles216,mix --reps 9 --so tools/variants/liblz4mi_pw2.so tools/variants/liblz4mi_pn1w2.so tools/variants/liblz4mi_po2.so > gpurun_out/prio/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/prio/ab.log; exit $rc
