#!/bin/bash
# SPH frame time under a tuning knob (run on the GPU box), after the SPH parity tests:
#   bash tools/sph_sweep.sh VAR "v1 v2 ..." [N ...]  -> gpurun_out/sph_sweep.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
var=$1; vals=$2; shift 2
sizes=${*:-65536 1048576 4194304}
timeout -k 10 300 python -u -m pytest tests/test_gpu_sph.py tests/test_gpu_golden.py tests/test_gpu_host_demo.py -q -x \
  --timeout 120 --timeout-method thread > gpurun_out/sph_tests.log 2>&1; rc=$?
tail -3 gpurun_out/sph_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/sph_sweep.log
for v in $vals; do
  for n in $sizes; do
    echo -n "$var=$v " >> gpurun_out/sph_sweep.log
    env "$var=$v" timeout -k 10 120 python3 tools/sph_frames.py $n 60 >> gpurun_out/sph_sweep.log 2>&1 || exit $?
  done
done
cat gpurun_out/sph_sweep.log
