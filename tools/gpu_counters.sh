# PMC instruction/wait/traffic counters of the batch encoder and the decoder (tiles216, 4096 x 4 MiB) -> gpurun_out/cnt4
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cnt4
timeout -k 10 900 bash tools/prof_counters.sh gpurun_out/cnt4/dec lz4mi_decompress_kernel -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 > gpurun_out/cnt4/dec.log 2>&1 || { echo dec failed; tail gpurun_out/cnt4/dec.log; exit 1; }
python tools/pmc_summary.py gpurun_out/cnt4/dec > gpurun_out/cnt4/pmc_counters_decode_tiles216.json
timeout -k 10 900 bash tools/prof_counters.sh gpurun_out/cnt4/comp lz4mi_compress_gts_kernel -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 --what compress > gpurun_out/cnt4/comp.log 2>&1 || { echo comp failed; tail gpurun_out/cnt4/comp.log; exit 1; }
python tools/pmc_summary.py gpurun_out/cnt4/comp > gpurun_out/cnt4/pmc_counters_compress_tiles216.json
cat gpurun_out/cnt4/pmc_counters_decode_tiles216.json gpurun_out/cnt4/pmc_counters_compress_tiles216.json
