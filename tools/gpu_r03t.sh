# decoder readlane-broadcast A/B + encoder miss-batch windows A/B (outputs checked)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03t
timeout -k 10 400 python -u tools/microbench.py --what compress --gens tiles216,random,mix --reps 3 --so tools/variants/liblz4mi_mwin.so > gpurun_out/r03t/comp.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03t/comp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/microbench.py --gens tiles216,mix,random --reps 7 --so tools/variants/liblz4mi_rl.so > gpurun_out/r03t/dec.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03t/dec.log; exit $rc
