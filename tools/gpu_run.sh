#!/bin/bash
# GPU-box driver for gpurun: runs the requested steps in order, each under its own time
# limit, logs under gpurun_out/.  A test *failure* (pytest rc 1) lets later steps run; any
# crash/abort/timeout (rc >= 2 from pytest, or != 0 from other steps) stops the script.
#   tools/gpu_run.sh tests smoke bench prof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
for step in "$@"; do
  case "$step" in
    tests)
      run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --durations=15 --timeout 300 --timeout-method thread; rc=$?
      [ $rc -le 1 ] || exit $rc ;;
    tests_sph)
      run pytest_gpu_sph 600 python -u -m pytest tests/test_gpu_sph.py tests/test_gpu_golden.py -m gpu -q -rf -x --timeout 120 --timeout-method thread; rc=$?
      [ $rc -le 1 ] || exit $rc ;;
    smoke)
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench)
      run bench 600 python bench.py || exit $? ;;
    bench_driver)
      run bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 || exit $? ;;
    prof_driver)
      run prof_driver 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_driver -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $? ;;
    bench_short)
      run bench_short 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline || exit $? ;;
    torchrun1)
      run torchrun1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 50 --warmup 10 --no-cpu-baseline || exit $? ;;
    prof)
      run prof_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline || exit $? ;;
    pmc)
      run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --allpairs-n 0 --sph-n 0 || exit $?
      run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --allpairs-n 0 --sph-n 0 || exit $? ;;
    prof_sph)
      run prof_sph 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sph -o run --output-format csv -- python3 tools/sph_frames.py 50000 60 || exit $? ;;
    prof_sph:*)
      n=${step#prof_sph:}
      run prof_sph_$n 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sph_$n -o run --output-format csv -- python3 tools/sph_frames.py $n 60 || exit $? ;;
    pmc_sph:*)
      # pmc_sph:N:C1,C2,...  one rocprofv3 --pmc pass (counters of one pass only) over SPH frames
      spec=${step#pmc_sph:}; n=${spec%%:*}; cs=${spec#*:}
      tag=$(echo "$cs" | tr ',' '\n' | head -1)
      run pmc_sph_${n}_$tag 120 rocprofv3 --kernel-trace --pmc ${cs//,/ } -d gpurun_out/pmc_sph_${n}_$tag -o run --output-format csv -- python3 tools/sph_frames.py $n 30 || exit $? ;;
    prof_sph64k)
      run prof_sph64k 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sph64k -o run --output-format csv -- python3 tools/sph_frames.py 65536 60 || exit $? ;;
    sizes)
      # SPH frame by size (all-active frames, tools/ab_sph.py, bench.py's window: 20 warm, 200
      # timed), one line per size
      for n in 20000 50000 65536 100000 262144 300000 1000000 1048576 2097152 4194304; do
        run sizes_$n 120 python tools/ab_sph.py --n $n --warm 20 --frames 200 --rounds 2 rust-particle-system_amd/lib/librps.so || exit $?
        grep "^n=" gpurun_out/sizes_$n.log >> gpurun_out/sizes.txt
      done ;;
    curve)
      run sph_frame_curve 300 python tools/sph_frame_curve.py || exit $? ;;
    probe)
      run hbm_probe 300 tools/hbm_probe || exit $? ;;
    *)
      # arbitrary python script under tools/: "py:tools/foo.py[,arg1,arg2...]"
      if [[ "$step" == py:* ]]; then
        IFS=, read -r -a pyargs <<< "${step#py:}"
        run "$(basename "${pyargs[0]}" .py)" 900 python "${pyargs[@]}" || exit $?
      else
        echo "unknown step $step"; exit 2
      fi ;;
  esac
done
