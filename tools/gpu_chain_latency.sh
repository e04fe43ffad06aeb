cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cl
for nb in 256 1024 2048 4096; do
  timeout -k 10 300 python -u tools/compress_ab.py --gens tiles216 --blocks $nb --enc "" --reps 2 >> gpurun_out/cl/chain.log 2>&1 || exit 1
  echo "blocks=$nb done" >> gpurun_out/cl/chain.log
done
cat gpurun_out/cl/chain.log
