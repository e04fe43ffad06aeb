# randomized encoder stress: LDS-table batches (<= 768 blocks) and global-table batches (> 768)
set -o pipefail
cd $GRAFT_REPO_ROOT && T=${1:-r05_encstress} && mkdir -p gpurun_out/$T
timeout -k 10 150 python -u tools/enc_fuzz.py --seconds 80 --seed 41 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/$T/enc.log || exit 1
timeout -k 10 150 python -u tools/enc_fuzz.py --seconds 80 --seed 42 --big 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/$T/enc.log || exit 1
