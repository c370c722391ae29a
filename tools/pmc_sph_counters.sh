#!/bin/bash
# Per-kernel counters of the 2^22 SPH frame for DESIGN.md §5.2's table (tools/sph_counter_table.py):
# a kernel trace (times), then two --pmc passes (each within one pass's counter limits:
# TCP 2, TA 1, SQ 3 / TCC 2, SQ 4) over tools/sph_frames.py, every frame active.
#   tools/pmc_sph_counters.sh [N]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
n=${1:-4194304}
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/cnt_trace_$n -o run --output-format csv -- python3 tools/sph_frames.py $n 40 > gpurun_out/cnt_trace_$n.log 2>&1 || { echo "trace failed rc=$?"; tail -20 gpurun_out/cnt_trace_$n.log; exit 1; }
echo "trace ok: $(grep ms/frame gpurun_out/cnt_trace_$n.log)"
pass() {
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/cnt_${tag}_$n -o run --output-format csv -- python3 tools/sph_frames.py $n 8 > gpurun_out/cnt_${tag}_$n.log 2>&1 || { echo "pmc $tag failed rc=$?"; tail -20 gpurun_out/cnt_${tag}_$n.log; exit 1; }
  echo "pmc $tag ok"
}
pass m1 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES
pass m2 TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
