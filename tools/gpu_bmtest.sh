set -o pipefail
mkdir -p gpurun_out/bm
LZ4MI_BITMAP=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/bm/pytest.log 2>&1 || { tail -30 gpurun_out/bm/pytest.log; exit 1; }
tail -1 gpurun_out/bm/pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LZ4MI_BITMAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bm/prof -o run --output-format csv -- python tools/microbench.py --gens tiles216 --blocks 4096 --reps 3 > gpurun_out/bm/prof.log 2>&1 || { tail gpurun_out/bm/prof.log; exit 1; }
grep tiles216 gpurun_out/bm/prof.log
head -6 $(find gpurun_out/bm/prof -name "*kernel_stats.csv") | cut -d, -f1-4
