#!/bin/bash
# Build a librps variant for same-box A/B runs: tools/build_variant.sh NAME KERNELS.hip [extra hipcc flags]
# -> ablibs/NAME/librps.so (rps_nbody.hip from the tree, the given kernels source, and the tree's
# rps_context.hip or $CTX_SRC).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; src=$2; shift 2
out=${AB_OUT:-$ROOT/ablibs}/$name
mkdir -p "$out"
cp "$src" "$ROOT/rust-particle-system_amd/csrc/.variant_$name.hip"
cp "${CTX_SRC:-$ROOT/rust-particle-system_amd/csrc/rps_context.hip}" "$ROOT/rust-particle-system_amd/csrc/.variant_ctx_$name.hip"
trap 'rm -f "$ROOT/rust-particle-system_amd/csrc/.variant_$name.hip" "$ROOT/rust-particle-system_amd/csrc/.variant_ctx_$name.hip"' EXIT
F="-std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -I$ROOT/include"
/opt/rocm/bin/hipcc $F "$@" -c -o "$out/k.o" "$ROOT/rust-particle-system_amd/csrc/.variant_$name.hip"
/opt/rocm/bin/hipcc $F -c -o "$out/c.o" "$ROOT/rust-particle-system_amd/csrc/.variant_ctx_$name.hip"
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-sched-strategy=max-ilp -c -o "$out/nb.o" "$ROOT/rust-particle-system_amd/csrc/rps_nbody.hip"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$out/librps.so" "$out/k.o" "$out/nb.o" "$out/c.o" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f "$out/k.o" "$out/c.o" "$out/nb.o"
echo "$out/librps.so"
