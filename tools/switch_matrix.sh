#!/bin/bash
# The SPH + golden GPU suites under each fallback switch (every path the defaults replace must stay
# bitwise): tools/switch_matrix.sh  -> gpurun_out/switch_matrix.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/switch_matrix.txt
: > "$out"
for sw in RPS_SPH_CSORT=0 RPS_SPH_PAIRS=0 RPS_SPH_SIM_FUSE=0 RPS_SPH_LONGQ=0 RPS_SPH_CSORT_WIDE=0 RPS_SPH_GROUP=2; do
  echo "== $sw" | tee -a "$out"
  env "$sw" timeout -k 10 300 python -u -m pytest tests/test_gpu_sph.py tests/test_gpu_golden.py -m gpu -q -x \
      --timeout 120 --timeout-method thread > gpurun_out/switch_run.log 2>&1
  rc=$?
  grep -E "passed|failed" gpurun_out/switch_run.log | tail -1 | tee -a "$out"
  [ $rc -le 1 ] || exit $rc
done
