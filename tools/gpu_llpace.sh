# long-literal copy depth / pacing variants on the mixes
cd $GRAFT_REPO_ROOT && T=${1:-r05c} && mkdir -p gpurun_out/$T
so=""; for v in d1 d2 d4s64 d4s127 d2s127; do so="$so tools/variants/liblz4mi_$v.so"; done
timeout -k 10 400 python -u tools/microbench.py --gens mix,mixc,random --reps 7 --so $so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_frames.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -5 | tee gpurun_out/$T/frames.log
