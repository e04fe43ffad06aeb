# A/B of two decoder builds (tools/variants/liblz4mi_$1.so vs _$2.so) in one process over generators $3.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
LZ4MI_DECODER=single timeout -k 10 400 python tools/microbench.py --gens ${3:-tiles216,mix,text,copy,runs} --blocks 4096 --reps 7 --skip-default --so tools/variants/liblz4mi_$1.so tools/variants/liblz4mi_$2.so > gpurun_out/ab/ab.json 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab/ab.json; exit 1; }
grep GBps gpurun_out/ab/ab.json
