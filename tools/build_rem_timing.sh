#!/bin/bash
# Build tools/bin/rem_timing.so: libppnp_amd.so with tools/rem_timing.patch applied to
# appnp_blocks.hip (per-wave real-time stamps in the remainder pass, read back by
# appnp_debug_rem_times). Diagnostic only; tools/rem_timing.py loads it via PPNP_AMD_LIB.
# Needs the main build first: make -C ppnp_amd/csrc
set -eu
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
mkdir -p "$tmp/ppnp_amd" "$root/tools/bin"
cp -r "$root/ppnp_amd/csrc" "$tmp/ppnp_amd/"
cp -r "$root/include" "$tmp/"
patch -s -d "$tmp" -p1 < "$root/tools/rem_timing.patch"
cp "$root"/ppnp_amd/csrc/build/*.o "$tmp/"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 \
  -c "$tmp/ppnp_amd/csrc/appnp_blocks.hip" -o "$tmp/appnp_blocks.o"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$root/tools/bin/rem_timing.so" "$tmp"/*.o -ldl
echo "built tools/bin/rem_timing.so"
