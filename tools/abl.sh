# counters for the default build and the parse-only ablation (tiles216)
tools/prof_counters.sh gpurun_out/pmc_cur lz4mi_decompress -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 > gpurun_out/pmc_cur.log 2>&1 || exit 1
tools/prof_counters.sh gpurun_out/pmc_ab1 lz4mi_decompress -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 --skip-default --so tools/variants/liblz4mi_ab1.so > gpurun_out/pmc_ab1.log 2>&1 || exit 1
