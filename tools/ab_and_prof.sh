# A/B microbench of tools/variants (except *_prof.so), then the phase profile of liblz4mi_prof.so
SOS="$(ls tools/variants/*.so | grep -v _prof.so)" GENS=${GENS:-tiles216,random,repetitive} bash tools/run_ab.sh || exit 1
if [ -f tools/variants/liblz4mi_prof.so ]; then
  timeout -k 10 300 python tools/phase_prof.py --blocks ${PBLOCKS:-4096} > gpurun_out/pp.log 2>&1; grep -v amdgpu gpurun_out/pp.log
fi
