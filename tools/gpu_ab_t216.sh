# tiles216 A/B of two decoder builds in one process, both orders.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
LZ4MI_DECODER=single timeout -k 10 300 python tools/microbench.py --gens tiles216,mix --blocks 4096 --reps 10 --skip-default --so tools/variants/liblz4mi_$1.so tools/variants/liblz4mi_$2.so tools/variants/liblz4mi_$1.so tools/variants/liblz4mi_$2.so > gpurun_out/ab/ab.json 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab/ab.json; exit 1; }
grep GBps gpurun_out/ab/ab.json
