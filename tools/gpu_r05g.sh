# frame decode in one launch (LZ4MI_FRAME_WORDS): frame tests, then the bench's mix-frame comparison
cd $GRAFT_REPO_ROOT && T=${1:-r05g} && mkdir -p gpurun_out/$T
true
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, 'divortio-lz4_amd'); import torch, json, lz4mi, bench
lz4mi.init(0)
s = torch.cuda.Stream(); torch.cuda.set_stream(s)
print(json.dumps(bench.mix_frame(torch, lz4mi, s, 2048)))
" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/mix_frame.log
