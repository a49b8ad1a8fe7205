#!/bin/bash
# Build a measurement variant of libppnp_amd.so into variants/<name>.so (git-ignored, but it
# travels to the GPU box with the tree): the listed sources recompiled with extra flags, the rest
# taken from the main build (make -C ppnp_amd/csrc).  Load it with PPNP_AMD_LIB=variants/<name>.so.
# Usage: tools/build_variant.sh <name> "<sources without .hip>" -DFLAG=1 ...
set -eu
name=$1; srcs=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/variants/obj-$name
mkdir -p "$out"
cp "$root"/ppnp_amd/csrc/build/*.o "$out/"
for f in $srcs; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" \
    -c "$root/ppnp_amd/csrc/$f.hip" -o "$out/$f.o" &
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$root/variants/$name.so" "$out"/*.o -ldl
rm -rf "$out"
echo "built variants/$name.so"
