#!/bin/bash
# Instruction counts of one kernel in a kernels source: tools/isa_count.sh SRC.hip KERNEL_SYMBOL_REGEX
# (device-only assembly for gfx950; VALU / SALU / LDS / global counts and the top opcodes).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
src=$1; pat=$2
tmp=$(mktemp -d)
cp "$src" "$ROOT/rust-particle-system_amd/csrc/.isa_tmp.hip"
trap 'rm -rf "$tmp" "$ROOT/rust-particle-system_amd/csrc/.isa_tmp.hip"' EXIT
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -ffp-contract=off -I"$ROOT/include" --cuda-device-only -S \
  -o "$tmp/k.s" "$ROOT/rust-particle-system_amd/csrc/.isa_tmp.hip" 2>&1 | grep -v "unused" || true
awk -v p="$pat" '$0 ~ "^"p".*:" && !f {f=1} f {print} f && /s_endpgm/ {exit}' "$tmp/k.s" > "$tmp/one.s"
printf "lines %s  valu %s  salu %s  lds %s  global %s\n" "$(wc -l < $tmp/one.s)" "$(grep -cE '^\s+v_' $tmp/one.s)" \
  "$(grep -cE '^\s+s_' $tmp/one.s)" "$(grep -cE '^\s+ds_' $tmp/one.s)" "$(grep -cE '^\s+global_' $tmp/one.s)"
grep -oE '^\s+[vsdg][a-z0-9_]+' "$tmp/one.s" | sort | uniq -c | sort -rn | head -${TOP:-12}
