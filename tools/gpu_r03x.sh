# dependent-block chain timings of the final build (tiles216, random, text, copy)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03x
timeout -k 10 500 python -u tools/chain_time.py tiles216,random,text > gpurun_out/r03x/chain.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03x/chain.log; exit $rc
