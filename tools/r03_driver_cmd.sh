#!/bin/bash
# Round 3: the driver's headline command (bench.py --gpus 1 --steps 20 --warmup 5) on one box,
# plain and under rocprofv3 --kernel-trace, beside the 500-step run, to see where the
# short run's extra time per step comes from (per-launch durations: tools/launch_series.py),
# and what bracketing every launch with HIP events costs (--profile-every 1 vs -1 / 8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03drv
export TMPDIR=/tmp
O=gpurun_out/r03drv
SIDE="--no-cpu-baseline --sph-n 0 --allpairs-n 0 --no-configs --export-reps 0"
show() { python3 -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$1',d['ms_per_step'],r.get('median_kernel_ms'),r.get('avg_kernel_ms'),r['launches'],r.get('profile_every'))"; }
for pe in 0 -1 8 0 -1; do
  f=$O/plain20_pe${pe}_$RANDOM.json
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --profile-every $pe $SIDE > $f 2> $f.err || exit $?
  show $f
done
echo "== rocprof driver command (full side runs)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof20 -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof20.json 2> $O/prof20.err || exit $?
show $O/prof20.json
echo "== rocprof 500/100"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof500 -o run --output-format csv -- python3 bench.py $SIDE > $O/prof500.json 2> $O/prof500.err || exit $?
show $O/prof500.json
echo "== plain 500/100"
timeout -k 10 240 python3 bench.py $SIDE > $O/plain500.json 2> $O/plain500.err || exit $?
show $O/plain500.json
echo "== plain 20/5 after the long runs"
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 $SIDE > $O/plain20_late.json 2> $O/plain20_late.err || exit $?
show $O/plain20_late.json
for f in $(find $O -name '*kernel_trace.csv'); do echo "== $f"; python3 tools/launch_series.py $f | tail -4; done
