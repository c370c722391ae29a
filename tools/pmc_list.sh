set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 60 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1; echo "list rc=$?"
grep -oE "SQ_[A-Z_0-9]+" gpurun_out/avail.txt | sort -u > gpurun_out/sq_avail.txt; wc -l gpurun_out/sq_avail.txt
