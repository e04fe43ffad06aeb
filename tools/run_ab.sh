# GPU tests, then A/B microbench of the default build against tools/variants/*.so
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1; tail -4 gpurun_out/t.log
timeout -k 10 400 python tools/microbench.py --gens ${GENS:-tiles216,random,repetitive} --blocks 4096 --reps 3 --so tools/variants/*.so > gpurun_out/mb.log 2>&1; grep -v amdgpu.ids gpurun_out/mb.log
