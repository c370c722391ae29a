#!/bin/bash
# Kernel trace of SPH frames per librps variant (run on the GPU box):
#   tools/ab_trace.sh N FRAMES PATTERN LIB...
# For each library: rocprofv3 --kernel-trace --stats over tools/ab_sph.py --one, then the
# stats lines whose kernel name matches PATTERN (grep -E).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abt
export TMPDIR=/tmp
n=$1; frames=$2; pat=$3; shift 3
i=0
for lib in "$@"; do
  i=$((i + 1))
  d=gpurun_out/abt/v$i
  echo "== $lib"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 ${AB_SCRIPT:-tools/sort_only.py} $lib $n $frames > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  tail -1 $d.log
  f=$(find $d -name '*kernel_stats.csv' | head -1)
  python3 tools/kstats.py $f > $d.stats
  grep -E "$pat" $d.stats || true
done
