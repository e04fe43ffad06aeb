# round-5 encoder: the table inserts as nontemporal stores (tabnt), and the table's zero-fill too
# (tabnt2), byte-identical check and time beside the default
cd $GRAFT_REPO_ROOT && T=${1:-r05q} && mkdir -p gpurun_out/$T
timeout -k 10 400 python -u tools/microbench.py --what compress --gens tiles216,mix,copy,random --reps 5 --so tools/variants/liblz4mi_tabnt.so tools/variants/liblz4mi_tabnt2.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/$T/tabnt.log
