timeout -k 10 120 tools/probe/store_bw > gpurun_out/sbw.log 2>&1; tail -3 gpurun_out/sbw.log
bash tools/prof_counters2.sh gpurun_out/sbwp "copies|memcpy|rows" "FETCH_SIZE,WRITE_SIZE,TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" -- tools/probe/store_bw && python tools/pmc_summary.py gpurun_out/sbwp
