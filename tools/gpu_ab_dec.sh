# decoder A/B of variant builds against the default (decoded bytes checked against the raw input)
#   tools/gpu_ab_dec.sh TAG GENS VARIANT...
cd $GRAFT_REPO_ROOT && T=$1 G=$2 && shift 2 && mkdir -p gpurun_out/$T
so=""; for v in "$@"; do so="$so tools/variants/liblz4mi_$v.so"; done
timeout -k 10 500 python -u tools/microbench.py --gens $G --reps 7 --so $so > gpurun_out/$T/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/$T/ab.log; exit $rc
