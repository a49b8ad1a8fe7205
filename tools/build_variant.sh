#!/bin/bash
# Build a measurement variant of libppnp_amd.so into tools/bin/<name>.so: the listed sources
# recompiled with extra flags, the rest taken from the main build (make -C ppnp_amd/csrc).
# Load it with PPNP_AMD_LIB=tools/bin/<name>.so.
# Usage: tools/build_variant.sh <name> "<sources without .hip>" -DFLAG=1 ...
set -eu
name=$1; srcs=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/tools/bin/$name
mkdir -p "$out"
cp "$root"/ppnp_amd/csrc/build/*.o "$out/"
for f in $srcs; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" \
    -c "$root/ppnp_amd/csrc/$f.hip" -o "$out/$f.o" &
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$root/tools/bin/$name.so" "$out"/*.o -ldl
rm -rf "$out"
echo "built tools/bin/$name.so"
