#!/bin/bash
# The oracle's CPU tests under AddressSanitizer + UndefinedBehaviorSanitizer (host code only;
# GPU sanitizers are not available on the pool).  Builds oracle/_asan/ and runs the tests
# that exercise the C restatement with the sanitizer runtimes preloaded into Python.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$ROOT/oracle" sanitize
export RPS_ORACLE_BUILD="$ROOT/oracle/_asan"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
cd "$ROOT"
exec python -m pytest -q -x -m "not gpu" -p no:cacheprovider tests/test_oracle_kat.py \
  tests/test_oracle_semantics.py tests/test_golden.py tests/test_wgsl_golden.py "$@"
