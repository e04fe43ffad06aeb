# Round-4 A/B: aligned periodic-run stores (decode), bulk emission on the LDS-permute build
# (encode), PCIe staging options for host-buffer calls.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04h
timeout -k 10 300 python -u tools/microbench.py --gens repetitive,random,tiles216 --reps 7 --so tools/variants/liblz4mi_peral.so > gpurun_out/r04h/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04h/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/microbench.py --what compress --gens tiles216,mix,text --reps 3 --so tools/variants/liblz4mi_bulk.so > gpurun_out/r04h/cab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04h/cab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/probe/pcie_staging.py > gpurun_out/r04h/pcie.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04h/pcie.log; exit $rc
