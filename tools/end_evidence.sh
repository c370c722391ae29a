#!/bin/bash
# End-of-round evidence in GPU calls of a few minutes each (every step under its own limit; the
# script stops at the first crash/timeout).  Outputs under gpurun_out/; tools/collect_profiles.py,
# tools/collect_sph_traffic.py and tools/sph_counter_table.py turn them into profiles/.
#   tools/end_evidence.sh a   smoke, the driver's bench command, its rocprofv3 kernel trace, the
#                             headline PMC passes (FETCH_SIZE, WRITE_SIZE: one per run)
#   tools/end_evidence.sh b   SPH traffic and counter passes at 2^22, the SPH frame curve at the
#                             reference's sizes, SPH frames by size (bench.py's window)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
case "${1:-}" in
  a) bash tools/gpu_run.sh smoke bench_driver prof_driver pmc || exit $? ;;
  b) bash tools/pmc_sph_traffic.sh || exit $?
     bash tools/pmc_sph_counters.sh 4194304 || exit $?
     bash tools/gpu_run.sh curve sizes || exit $? ;;
  *) echo "usage: $0 a|b"; exit 2 ;;
esac
