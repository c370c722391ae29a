#!/bin/bash
# SQ stall counters of the SPH kernels at N particles (one --pmc pass per group of at most 8 SQ
# counters, each kept only if this box's rocprofv3 lists it): tools/pmc_sq.sh N [LIB]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
n=$1; lib=${2:-rust-particle-system_amd/lib/librps.so}
timeout -k 5 60 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1
pass() {
  local tag=$1; shift
  local cs=()
  for c in "$@"; do grep -q "\b$c\b" gpurun_out/avail.txt && cs+=("$c"); done
  echo "pass $tag: ${cs[*]}"
  [ ${#cs[@]} -gt 0 ] || return 0
  AB_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "${cs[@]}" -d gpurun_out/sq_$tag -o run --output-format csv -- python3 tools/sph_frames.py $n 8 > gpurun_out/sq_$tag.log 2>&1 || { echo "pass $tag rc=$?"; tail -5 gpurun_out/sq_$tag.log; exit 1; }
}
pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA
pass b SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES
pass c SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F32
