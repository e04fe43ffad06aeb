# PMC counters of the ring decoder on tiles216 (separate rocprofv3 passes).
set -o pipefail
O=gpurun_out/${1:-pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $O
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_LDS_UNALIGNED_STALL" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-include-regex "${KRE:-ring_decode|token_map}" --pmc $pmc -d "$O/p$i" -o pmc --output-format csv -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 1 > "$O/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python tools/pmc_summary.py $O
