#!/bin/bash
# Round-4 GPU step: decoder parity tests (+ optional extra test files), then the decode A/B
# microbench of the default build against the given variants.
#   tools/gpu_r04.sh TAG "TESTS" GENS VARIANT...
set -o pipefail
T=$1; TESTS=$2; G=$3; shift 3
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$T
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu $TESTS > gpurun_out/$T/pytest.log 2>&1
  rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/$T/pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
fi
so=""; for v in "$@"; do so="$so tools/variants/liblz4mi_$v.so"; done
timeout -k 10 500 python -u tools/microbench.py --gens $G --reps 7 ${so:+--so $so} > gpurun_out/$T/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/$T/ab.log; exit $rc
