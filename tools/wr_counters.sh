# write-path counters of the decoder (tiles216, 4096 blocks) and of the store probes
S="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITE_sum TCC_WRITEBACK_sum,TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCC_EA0_WRREQ_STALL_sum,TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_WRITE_SECTORS_sum TCC_STREAMING_REQ_sum GRBM_GUI_ACTIVE"
bash tools/prof_counters2.sh gpurun_out/wrd lz4mi_decompress_kernel "$S" -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 && python tools/pmc_summary.py gpurun_out/wrd && \
bash tools/prof_counters2.sh gpurun_out/wrp "rows|runs|memcpy_runs" "$S" -- tools/probe/store_bw && python tools/pmc_summary.py gpurun_out/wrp
