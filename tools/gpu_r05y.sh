# round-5 small-batch decode in reference mode (LZ4MI_JS_EXACT: F1 check + batch-kernel redo of
# the blocks it changes): the whole GPU suite (JS-exact tests now take the small path), latency
cd $GRAFT_REPO_ROOT && T=${1:-r05y} && mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tests.log || exit 1
timeout -k 10 300 python -u tools/small_latency.py --js-exact --gens tiles216,text,copy 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/latency_js.log || exit 1
LZ4MI_SMALL_BLOCKS=0 timeout -k 10 300 python -u tools/small_latency.py --js-exact --gens tiles216,text,copy --counts 1,16 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/latency_js_batch.log || exit 1
