# encoder: scattered emission A/B (byte-identity checked against the default build)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03y
timeout -k 10 400 python -u tools/microbench.py --what compress --gens tiles216,random,mix --reps 3 --so tools/variants/liblz4mi_sc.so > gpurun_out/r03y/comp.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03y/comp.log; exit $rc
