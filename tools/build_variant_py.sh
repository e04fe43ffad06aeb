#!/bin/bash
# Like build_variant.sh, but the edit is a python script run on a copy of the
# decoder source (argv[1] of the script = the file to edit).
#   tools/build_variant_py.sh NAME edit.py [extra hipcc flags]
set -e
name=$1; py=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/divortio-lz4_amd/csrc
T=$(mktemp -d)
cp $C/*.h $C/*.hip $C/*.cpp $T/
F0=${FILE:-lz4mi_decompress.hip}
python3 "$py" $T/$F0
mkdir -p $R/tools/variants
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include $*"
objs=""
for f in lz4mi_decompress.hip lz4mi_expand.hip lz4mi_decompress_serial.hip lz4mi_compress.hip lz4mi_xxh32.hip lz4mi_frame.hip lz4mi_capi.cpp; do
  if [ "$f" = "$F0" ]; then srcf=$T/$f; else srcf=$C/$f; fi
  /opt/rocm/bin/hipcc $F -c -o $T/$f.o $srcf & objs="$objs $T/$f.o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $R/tools/variants/liblz4mi_$name.so $objs
rm -rf $T
echo built tools/variants/liblz4mi_$name.so
