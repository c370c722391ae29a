#!/bin/bash
# Round 3: GPU tests, then the static-network tail sort launch A/B (ablibs/base vs ablibs/tail)
# at the three sort tile sizes, then a kernel trace of the 2^22 SPH frames.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 4194304 1048576 524288; do
  echo "== ab n=$n"
  timeout -k 10 300 python3 tools/ab_sph.py --n $n --frames 50 --rounds 3 ablibs/base/librps.so ablibs/tail/librps.so ablibs/pairs/librps.so ablibs/head/librps.so > gpurun_out/ab_sort_$n.log 2>&1 || { cat gpurun_out/ab_sort_$n.log; exit 1; }
  cat gpurun_out/ab_sort_$n.log
done
echo "== prof sph 2^22"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sph_r03 -o run --output-format csv -- python3 tools/sph_frames.py 4194304 60 > gpurun_out/prof_sph_r03.log 2>&1 || exit 1
find gpurun_out/prof_sph_r03 -name '*kernel_stats.csv' | head -1 | xargs python3 tools/kstats.py | head -30
