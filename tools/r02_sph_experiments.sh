#!/bin/bash
# Round-2 SPH experiments in one GPU call (each step under its own time limit; the first
# failure ends the script).  Logs under gpurun_out/.
#   1. bitwise parity with the later local sort launches on 4096-entry tiles (RPS_SORT_TILE2)
#   2. same-box frame times: sort tile2, sim output scatter variants, split sim
#   3. frozen-state probes: the sim / density with trivial bodies (same loads, same masks)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=rust-particle-system_amd/lib/librps.so
RPS_SORT_TILE2=4096 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_sph.py -k "bench_workload or large_frames or steps_bitwise" > gpurun_out/x_tile2_tests.log 2>&1
timeout -k 10 400 python -u tools/ab_sph.py --n 4194304 --frames 50 --rounds 3 $L $L@RPS_SORT_TILE2=4096 \
  $L@RPS_SORT_TILE2=2048 ablibs/simslot/librps.so ablibs/simpref/librps.so ablibs/split/librps.so \
  > gpurun_out/x_ab_22.log 2>&1
timeout -k 10 300 python -u tools/ab_sph.py --n 1048576 --frames 100 --rounds 3 $L $L@RPS_SORT_TILE2=2048 \
  ablibs/split/librps.so > gpurun_out/x_ab_20.log 2>&1
timeout -k 10 300 python -u tools/ab_sph.py --n 4194304 --frames 50 --rounds 3 ablibs/frozen/librps.so \
  ablibs/frozen_simprobe/librps.so ablibs/frozen_denprobe/librps.so > gpurun_out/x_ab_frozen.log 2>&1
echo done
