#!/bin/bash
# SQ counters of the SPH frame kernels (one --pmc pass per run, counters per kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD \
    -d gpurun_out/pmc_sph_$n -o run --output-format csv -- python3 tools/sph_frames.py $n 12 > gpurun_out/pmc_sph_$n.log 2>&1 || { echo "pmc $n failed rc=$?"; tail -20 gpurun_out/pmc_sph_$n.log; exit 1; }
  echo "pmc $n ok"
done
