#!/bin/bash
# Round 5: packed-lookup sort -- SPH GPU suites (packed path at 2^21-2^22), then 2^22 / 2^21 traces
# with and without RPS_SPH_SORT_PACK.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sph.py tests/test_gpu_golden.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t_sph.log 2>&1; rc=$?; tail -3 gpurun_out/t_sph.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_variants.sh 4194304 30 pack=tree nopack=tree@RPS_SPH_SORT_PACK=0 || exit $?
bash tools/prof_variants.sh 2097152 30 pack=tree nopack=tree@RPS_SPH_SORT_PACK=0 || exit $?
