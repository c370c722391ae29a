#!/bin/bash
# Round-5 end-of-round evidence in one GPU call (each step under its own limit; stops at the
# first crash/timeout): the GPU suite and smoke, the driver's bench command and its rocprofv3
# kernel trace, the headline PMC passes (FETCH_SIZE, WRITE_SIZE: one per run), the SPH traffic
# passes, and SPH frames by size.  Outputs under gpurun_out/ (tools/collect_*.py copy them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_run.sh tests smoke bench_driver prof_driver pmc || exit $?
bash tools/pmc_sph_traffic.sh || exit $?
bash tools/gpu_run.sh sizes || exit $?
