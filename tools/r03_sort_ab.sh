#!/bin/bash
# Round 3: same-box A/B of the SPH frame over librps variants (tools/ab_sph.py), then a kernel
# trace of the 2^22 SPH frames with the tree's library.
#   tools/r03_sort_ab.sh "N1 N2 ..." VARIANT...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
sizes=$1; shift
for n in $sizes; do
  echo "== ab n=$n"
  timeout -k 10 400 python3 tools/ab_sph.py --n $n --frames 50 --rounds 2 "$@" > gpurun_out/ab_sort_$n.log 2>&1 || { cat gpurun_out/ab_sort_$n.log; exit 1; }
  cat gpurun_out/ab_sort_$n.log
done
echo "== prof sph 2^22"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sph_r03 -o run --output-format csv -- python3 tools/sph_frames.py 4194304 60 > gpurun_out/prof_sph_r03.log 2>&1 || exit 1
find gpurun_out/prof_sph_r03 -name '*kernel_stats.csv' | head -1 | xargs python3 tools/kstats.py | head -40
