#!/bin/bash
# Like prof_counters.sh with the counter passes given as arguments separated by ','
#   tools/prof_counters2.sh OUTDIR KERNEL_REGEX "A B,C D" -- cmd ...
set -o pipefail
OUT=$1; KRE=$2; SETS=$3; shift 3; [ "$1" = "--" ] && shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
i=0
IFS=',' read -ra PASSES <<< "$SETS"
for pmc in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-include-regex "$KRE" --pmc $pmc -d "$OUT/p$i" -o pmc --output-format csv -- "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
