# tiles216/mix A/B of three decoder builds in one process, interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
V=tools/variants/liblz4mi_
LZ4MI_DECODER=single timeout -k 10 400 python tools/microbench.py --gens ${4:-tiles216,mix} --blocks 4096 --reps 9 --skip-default --so $V$1.so $V$2.so $V$3.so > gpurun_out/ab/ab3.json 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab/ab3.json; exit 1; }
grep GBps gpurun_out/ab/ab3.json
