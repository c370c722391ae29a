#!/bin/bash
# The driver's headline command three times on one box (ms/step beside the kernel average).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/drv3
export TMPDIR=/tmp
for rep in 1 2 3; do
  o=gpurun_out/drv3/drv_$rep.json
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sph-n 0 --allpairs-n 0 > $o 2> $o.err || { tail -5 $o.err; exit 1; }
  python3 -c "import json;d=json.load(open('$o'));r=d['roofline'];print($rep, d['value'], round(d['ms_per_step'],4), round(r['avg_kernel_ms'],4))"
done
