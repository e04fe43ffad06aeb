mkdir -p gpurun_out
for nb in 1024 2048 4096 8192; do timeout -k 10 300 python tools/microbench.py --gens tiles216 --blocks $nb --reps 3 > gpurun_out/nb$nb.log 2>&1 || exit 1; grep tiles gpurun_out/nb$nb.log; done
timeout -k 10 900 bash tools/prof_counters.sh gpurun_out/pc lz4mi_decompress_kernel -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 && python tools/pmc_summary.py gpurun_out/pc > gpurun_out/pc.json && cat gpurun_out/pc.json
