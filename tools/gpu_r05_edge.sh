# the window-edge offset fix: the new test against the pre-fix library (must fail) and the fixed one,
set -o pipefail
# the GPU suite, the fuzz-found block in every re-parse mode, the small-path stress in every mode
cd $GRAFT_REPO_ROOT && T=${1:-r05_edge} && mkdir -p gpurun_out/$T
timeout -k 10 120 python -u tools/run_test_with_so.py tools/variants/liblz4mi_prefix.so test_sequence_ending_on_the_window_edge 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/old_lib.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tests.log || exit 1
for m in 0 1 2; do LZ4MI_SMALL_REPARSE=$m timeout -k 10 100 python -u tools/small_repro.py tools/variants/mismatch_d1.npz 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/$T/repro.log || exit 1; done
for m in 0 1 2; do LZ4MI_SMALL_REPARSE=$m timeout -k 10 150 python -u tools/small_fuzz.py --seconds 50 --seed $((20 + m)) --dump gpurun_out/$T/d$m 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/$T/fuzz.log || exit 1; done
