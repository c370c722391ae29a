#!/bin/bash
# Round 3: the driver's headline command with the side runs after (default) or before the
# headline, alternated on one box (tools/r03_order_test.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/order
export TMPDIR=/tmp
for rep in 1 2; do
  for v in none configs "configs,sph" "allpairs,sph,configs"; do
    o=gpurun_out/order/${v//,/_}_$rep.json
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sides-first "$v" > $o 2> $o.err || { echo "fail $v"; tail -5 $o.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('$o'));print('$v', $rep, round(d['ms_per_step'],4), round(d['roofline']['avg_kernel_ms'],4))"
  done
done
