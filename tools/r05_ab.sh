#!/bin/bash
# Round 5 A/B driver: SPH GPU suites on the tree, then kernel traces of the tree vs abx/old at the
# given sizes: tools/r05_ab.sh N1 N2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sph.py tests/test_gpu_golden.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t_sph.log 2>&1; rc=$?; tail -3 gpurun_out/t_sph.log; [ $rc -eq 0 ] || exit $rc
for n in "$@"; do
  bash tools/prof_variants.sh $n 40 new=tree old=abx/old/librps.so ${AB_EXTRA:-} || exit $?
done
