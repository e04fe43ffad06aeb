# round-5 encoder: what a table write-back costs by its width -- shadow copies of every table
# insert as a 2-byte store (shadow), nontemporal 2-byte (shnt), one aligned 16-byte store
# (sh16), four covering an aligned 64 bytes (sh64); time beside the default, WRITE_SIZE of sh16/sh64
cd $GRAFT_REPO_ROOT && T=${1:-r05p} && mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/microbench.py --what compress --gens tiles216,mix --reps 3 --so tools/variants/liblz4mi_shadow.so tools/variants/liblz4mi_shnt.so tools/variants/liblz4mi_sh16.so tools/variants/liblz4mi_sh64.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/shadow_width.log || exit 1
for v in sh16 sh64 shnt; do
timeout -k 10 300 rocprofv3 --kernel-include-regex lz4mi_compress_gts_kernel --pmc WRITE_SIZE -d gpurun_out/$T/pmc_$v -o pmc \
  --output-format csv -- python tools/microbench.py --what compress --gens tiles216 --blocks 4096 --reps 1 --so tools/variants/liblz4mi_$v.so --skip-default > gpurun_out/$T/pmc_$v.log 2>&1 || { echo "pass failed"; exit 1; }
echo pass $v ok
done
