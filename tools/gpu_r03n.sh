# compress PMC traffic of the current build + phase profile of the batch encoder
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03n
timeout -k 10 600 bash tools/pmc_traffic.sh gpurun_out/r03n/pmc_c tiles216 compress > gpurun_out/r03n/pmc_c.log 2>&1 || { echo pmc compress failed; tail -5 gpurun_out/r03n/pmc_c.log; exit 1; }
tail -14 gpurun_out/r03n/pmc_c.log
timeout -k 10 300 python -u tools/gts_prof.py --gens tiles216,random,text > gpurun_out/r03n/cprof.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03n/cprof.log; exit $rc
