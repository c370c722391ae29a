#!/bin/bash
# Memory-pipeline counters of the SPH frame kernels at N particles (one --pmc pass per run).
#   tools/pmc_sph_mem.sh N "COUNTERS..." TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
n=$1; ctr=$2; tag=$3
timeout -s KILL 90 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${tag}_$n -o run --output-format csv -- python3 tools/sph_frames.py $n 12 > gpurun_out/pmc_${tag}_$n.log 2>&1 || { echo "pmc $tag $n failed rc=$?"; tail -20 gpurun_out/pmc_${tag}_$n.log; exit 1; }
echo "pmc $tag $n ok"
