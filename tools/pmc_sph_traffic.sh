#!/bin/bash
# Measured traffic behind the SPH roofline (round 3): three separate rocprofv3 --pmc passes over
# tools/sph_traffic_frames.py (a calibration stream, then the bench's 2^22 SPH frames):
# FETCH_SIZE, WRITE_SIZE (memory side) and the L1 -> L2 request counts.  Each pass its own run
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share one).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/$name -o run --output-format csv -- python3 tools/sph_traffic_frames.py 4194304 12 > gpurun_out/$name.log 2>&1 || { echo "pmc $name failed rc=$?"; tail -20 gpurun_out/$name.log; exit 1; }
  echo "pmc $name ok"
}
pass pmc_sph_fetch FETCH_SIZE
pass pmc_sph_write WRITE_SIZE
pass pmc_sph_l2req TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
