#!/bin/bash
# Build an A/B variant of libfia.so: the in-tree objects with ONE unit recompiled from a modified
# copy of its source.  usage: tools/build_variant.sh <unit (e.g. gram_mf)> <modified .hip> <out.so>
set -eu
cd "$(dirname "$0")/.."
unit=$1; src=$2; out=$3
C=fia-kdd-19_amd/csrc
make -C $C -j8 >/dev/null
tmp=$(mktemp -d)
cp $C/*.h "$tmp/"
cp "$src" "$tmp/$unit.hip"
extra=""
[ "$unit" = gram_mf ] && extra="-mllvm -amdgpu-mfma-vgpr-form"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Wall -Wno-unused-function -Wno-unused-result \
  -munsafe-fp-atomics -mllvm -pragma-unroll-threshold=200000 $extra -c "$tmp/$unit.hip" -o "$tmp/$unit.o"
objs=""
for o in $C/build/*.o; do b=$(basename "$o" .o); [ "$b" = "$unit" ] && objs="$objs $tmp/$unit.o" || objs="$objs $o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o "$out"
rm -rf "$tmp"
echo "built $out"
