# encoder window-refill threshold A/B (byte-identity checked against the default build)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03o
timeout -k 10 500 python -u tools/microbench.py --what compress --gens tiles216,random --reps 3 --so tools/variants/liblz4mi_rf128.so tools/variants/liblz4mi_rf32.so tools/variants/liblz4mi_rf256m.so > gpurun_out/r03o/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03o/ab.log; exit $rc
