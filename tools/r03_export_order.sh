#!/bin/bash
# Round 3: the driver's headline command with the export side measurement before the warmup
# (default) or after the timed region (--export-after), alternated on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/exo
export TMPDIR=/tmp
SIDE="--no-cpu-baseline --sph-n 0 --allpairs-n 0"
for rep in 1 2 3; do
  for v in before after; do
    o=gpurun_out/exo/${v}_$rep.json
    extra=""; [ $v = after ] && extra="--export-after"
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 $SIDE $extra > $o 2> $o.err || { echo "fail $v"; tail -5 $o.err; exit 1; }
    python3 -c "import json;d=json.load(open('$o'));print('$v', $rep, round(d['ms_per_step'],4), round(d['roofline']['avg_kernel_ms'],4), round(d['export']['ms_per_export'],4))"
  done
done
