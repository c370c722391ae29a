#!/bin/bash
# Kernel traces of SPH frames under several librps builds on one box:
#   tools/prof_variants.sh N FRAMES NAME=LIB ...   (LIB "tree": the in-tree build)
# -> gpurun_out/pv_<N>_<NAME>/ (rocprofv3 --kernel-trace --stats) and a compact table per build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
n=$1; frames=$2; shift 2
for spec in "$@"; do
  name=${spec%%=*}; lib=${spec#*=}
  envset=""
  case "$lib" in *@*) envset=${lib#*@}; lib=${lib%%@*} ;; esac  # NAME=LIB@VAR=VAL
  [ "$lib" = tree ] && lib=rust-particle-system_amd/lib/librps.so
  d=gpurun_out/pv_${n}_$name
  [ -n "$envset" ] && export "$envset"
  AB_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tools/sph_frames.py $n $frames > $d.log 2>&1
  rc=$?
  [ -n "$envset" ] && unset "${envset%%=*}"
  echo "== $name rc=$rc $(grep 'ms/frame' $d.log)"
  [ $rc -eq 0 ] || exit $rc
  python3 tools/kstats.py $(find $d -name '*kernel_stats.csv' | head -1) > $d.kstats; head -24 $d.kstats
done
