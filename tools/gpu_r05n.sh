# round-5 encoder questions: (1) the 15-bit table in LDS on the current
# hit-batch design (3 blocks per CU), 4096 blocks and one resident round of 768; (2) where the
# writes go: WRITE_SIZE of the default build against a build that repeats every table store
# into the never-read upper half of the block's table slot (the difference = the table stores'
# write-backs); FETCH_SIZE of the default build
cd $GRAFT_REPO_ROOT && T=${1:-r05n} && mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/microbench.py --what compress --gens tiles216,mix --reps 3 --so tools/variants/liblz4mi_ldst.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/ldst_4096.log || exit 1
timeout -k 10 300 python -u tools/microbench.py --what compress --gens tiles216 --blocks 768 --reps 3 --so tools/variants/liblz4mi_ldst.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/ldst_768.log || exit 1
for v in default shadow; do
  so=""; [ $v = shadow ] && so="--so tools/variants/liblz4mi_shadow.so --skip-default"
  for pmc in WRITE_SIZE FETCH_SIZE; do
    [ $v = shadow ] && [ $pmc = FETCH_SIZE ] && continue
    timeout -k 10 300 rocprofv3 --kernel-include-regex lz4mi_compress_gts_kernel --pmc $pmc -d gpurun_out/$T/pmc_$v/$pmc -o pmc \
      --output-format csv -- python tools/microbench.py --what compress --gens tiles216 --blocks 4096 --reps 1 $so > gpurun_out/$T/pmc_${v}_$pmc.log 2>&1 || { echo "pass $v $pmc failed"; exit 1; }
    echo "pass $v $pmc ok"
  done
done
