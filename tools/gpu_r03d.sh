cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03d
timeout -k 10 300 python -u tools/chain_time.py tiles216,text,random > gpurun_out/r03d/chain.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03d/chain.log
STEPS="tests bench" bash tools/gpu_round.sh r03d
