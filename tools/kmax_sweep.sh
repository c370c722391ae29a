#!/bin/bash
# SPH frame time across sort-knob variants on the GPU box, after the SPH parity tests run
# under each variant.  A variant is comma-separated env assignments ("-" = defaults):
#   bash tools/kmax_sweep.sh "RPS_SORT_TILE=4096 RPS_SORT_TILE=4096,RPS_SORT_KMAX=3 -" "n1 n2 ..."
#   -> gpurun_out/knob_sweep.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
variants=$1; sizes=${2:-65536 1048576 4194304}
for v in $variants; do
  IFS=, read -r -a kv <<< "${v/#-/RPS_NONE=1}"
  env "${kv[@]}" timeout -k 10 300 python -u -m pytest tests/test_gpu_sph.py -q -x --timeout 120 \
    --timeout-method thread > gpurun_out/sph_tests_knob.log 2>&1 || { tail -30 gpurun_out/sph_tests_knob.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/sph_tests_knob.log)"
done
: > gpurun_out/knob_sweep.log
for rep in 1 2; do
  for v in $variants; do
    IFS=, read -r -a kv <<< "${v/#-/RPS_NONE=1}"
    for n in $sizes; do
      echo -n "$v " >> gpurun_out/knob_sweep.log
      env "${kv[@]}" timeout -k 10 120 python3 tools/sph_frames.py $n 200 >> gpurun_out/knob_sweep.log 2>&1 || exit 1
    done
  done
done
cat gpurun_out/knob_sweep.log
