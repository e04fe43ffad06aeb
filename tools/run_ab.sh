for nb in 256 4096; do
timeout -k 10 300 python tools/microbench.py --gens tiles216 --blocks $nb --reps 3 --so tools/variants/liblz4mi_ab4.so tools/variants/liblz4mi_ab5.so tools/variants/liblz4mi_ab6.so 2>&1 | grep -v amdgpu.ids || exit 1
done
