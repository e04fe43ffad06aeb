#!/bin/bash
# instruction-cache / issue counters for one command (separate pass)
OUT=$1; shift; [ "$1" = "--" ] && shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-include-regex lz4mi_decompress --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU -d "$OUT/p1" -o pmc --output-format csv -- "$@" > "$OUT/p1.log" 2>&1
