#!/bin/bash
# Build an alternative liblz4mi.so from the current sources with a sed edit
# applied to the decoder (A/B timing with tools/microbench.py --so).
#   tools/build_variant.sh NAME 'sed-expr' [extra hipcc flags]
# FILE=lz4mi_compress.hip applies the edit to the encoder instead.
set -e
name=$1; expr=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/divortio-lz4_amd/csrc
T=$(mktemp -d)
cp $C/*.h $C/*.hip $C/*.cpp $T/
F0=${FILE:-lz4mi_decompress.hip}
[ -n "$SRCFILE" ] && cp "$SRCFILE" $T/$F0   # a whole replacement source for $F0 (e.g. from git show)
sed -i "$expr" $T/$F0
sed -i 's|"../../include/lz4mi.h"|"lz4mi.h"|' $T/*.hip $T/*.cpp $T/*.h   # (the copies sit outside the tree)
mkdir -p $R/tools/variants
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include $*"
objs=""
for f in lz4mi_decompress.hip lz4mi_expand.hip lz4mi_decompress_serial.hip lz4mi_compress.hip lz4mi_xxh32.hip lz4mi_frame.hip lz4mi_capi.cpp lz4mi_host.cpp; do
  srcf=$T/$f
  /opt/rocm/bin/hipcc $F -c -o $T/$f.o $srcf & objs="$objs $T/$f.o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $R/tools/variants/liblz4mi_$name.so $objs
rm -rf $T
echo built tools/variants/liblz4mi_$name.so
