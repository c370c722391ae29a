#!/bin/bash
# Round 3: the driver's headline command (bench.py --gpus 1 --steps 20 --warmup 5) on one box,
# plain and under rocprofv3 --kernel-trace, beside the 500-step run, to see where the
# short run's extra time per step comes from (per-launch durations: tools/launch_series.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03drv
export TMPDIR=/tmp
O=gpurun_out/r03drv
SIDE="--no-cpu-baseline --sph-n 0 --allpairs-n 0 --no-configs --export-reps 0"
for i in 1 2 3; do
  echo "== plain 20/5 #$i"
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 $SIDE > $O/plain20_$i.json 2> $O/plain20_$i.err || exit $?
  python3 -c "import json;d=json.load(open('$O/plain20_$i.json'));print(d['ms_per_step'],d['roofline']['avg_kernel_ms'],d['roofline']['launches'])"
done
echo "== rocprof driver command (full side runs)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof20 -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof20.json 2> $O/prof20.err || exit $?
echo "== rocprof 500/100"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof500 -o run --output-format csv -- python3 bench.py $SIDE > $O/prof500.json 2> $O/prof500.err || exit $?
echo "== plain 500/100"
timeout -k 10 240 python3 bench.py $SIDE > $O/plain500.json 2> $O/plain500.err || exit $?
python3 -c "import json;d=json.load(open('$O/plain500.json'));print(d['ms_per_step'],d['roofline']['avg_kernel_ms'],d['roofline']['launches'])"
echo "== plain 20/5 after the long runs"
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 $SIDE > $O/plain20_late.json 2> $O/plain20_late.err || exit $?
python3 -c "import json;d=json.load(open('$O/plain20_late.json'));print(d['ms_per_step'],d['roofline']['avg_kernel_ms'],d['roofline']['launches'])"
find $O -name '*kernel_trace.csv' -o -name '*kernel_stats.csv'
