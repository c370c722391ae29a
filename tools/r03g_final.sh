#!/bin/bash
# Round 3 final-tree measurement: the default bench line, the driver's command twice, and a
# kernel trace of the driver's command (export before the warmup).  Each GPU
# step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r03h}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > $O/$name.out 2> $O/$name.err || { echo "$name failed rc=$?"; tail -20 $O/$name.err; exit 1; }; }
step bench_default 400 python3 bench.py
step drv20_a 240 python3 bench.py --gpus 1 --steps 20 --warmup 5
step drv20_b 240 python3 bench.py --gpus 1 --steps 20 --warmup 5
step prof_drv20 400 rocprofv3 --kernel-trace --stats -d $O/prof_drv20 -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
step prof_sph 300 rocprofv3 --kernel-trace --stats -d $O/prof_sph -o run --output-format csv -- python3 tools/sph_frames.py 4194304 60
for f in bench_default drv20_a drv20_b prof_drv20; do python3 -c "import json;d=json.load(open('$O/$f.out'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r['avg_kernel_ms'],r['frac'],r['moved_frac'],d.get('sph',{}).get('ms_per_frame'),d.get('allpairs',{}).get('roofline',{}).get('frac_at_sustained_clock'))"; done
