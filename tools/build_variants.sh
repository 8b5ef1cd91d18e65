#!/bin/bash
# Builds kernel variants (compile-time knobs of trace.hip) as separate shared libraries under
# gpu-ray_trace-rust_amd/lib/variants/ for A/B timing in one process (tools/variant_bench.py).
# Usage: tools/build_variants.sh name1="-DKNOB=1 ..." name2="..."
set -e
PKG=$(dirname "$0")/../gpu-ray_trace-rust_amd
cd "$PKG"
make -s build/kd_build.o build/mesh_flatten.o build/doc.o build/pack.o build/scheme_host.o
mkdir -p lib/variants build/variants
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-rdc -munsafe-fp-atomics"
for spec in "$@"; do
  name=${spec%%=*}; defs=${spec#*=}
  hipcc $FLAGS -fno-slp-vectorize $defs -c -o build/variants/trace_$name.o csrc/kernel/${SRC:-trace.hip} &
  hipcc $FLAGS $defs -c -o build/variants/runtime_$name.o csrc/host/runtime.hip &
  wait
  hipcc --offload-arch=gfx950 -shared -o lib/variants/librt_$name.so build/kd_build.o build/mesh_flatten.o build/doc.o build/pack.o build/scheme_host.o build/variants/runtime_$name.o build/variants/trace_$name.o -lz
  echo "built $name: $defs"
done
