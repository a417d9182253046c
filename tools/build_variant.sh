#!/bin/bash
# Build an experiment variant of the engine: tools/build_variant.sh OUT.so "-DMACRO=V ..."
# (the in-tree objects are untouched; the variant links its own objects under /tmp)
set -eu
cd "$(dirname "$0")/.."
out=$1; defs=$2
tmp=$(mktemp -d)
objs=()
for s in lfe_capi lfe_prep lfe_sweep lfe_fast lfe_iter lfe_seg lfe_gram lfe_cluster lfe_keys lfe_compress lfe_synth; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -fno-gpu-rdc -w \
    -I/opt/rocm/include $defs -c leanfe_amd/csrc/$s.hip -o $tmp/$s.o &
  objs+=($tmp/$s.o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 "${objs[@]}" -o "$out" -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$tmp"
echo "built $out ($defs)"
