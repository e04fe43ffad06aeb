# PMC instruction/wait counters of the batch encoder and the single-pass decoder (tiles216, 4096 x 4 MiB)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cnt
timeout -k 10 900 bash tools/prof_counters.sh gpurun_out/cnt/comp lz4mi_compress_gt_kernel -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 --what compress > gpurun_out/cnt/comp.log 2>&1 || { echo comp failed; tail gpurun_out/cnt/comp.log; exit 1; }
timeout -k 10 900 bash tools/prof_counters.sh gpurun_out/cnt/dec lz4mi_decompress_kernel -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 > gpurun_out/cnt/dec.log 2>&1 || { echo dec failed; tail gpurun_out/cnt/dec.log; exit 1; }
echo ok
