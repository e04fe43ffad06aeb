# round pass of the current build, then the next-batch table prefetch A/B
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh r03w || exit $?
bash tools/gpu_r03v.sh
