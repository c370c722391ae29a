set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 5 60 tools/xlane_check > gpurun_out/xlane.log 2>&1; rc=$?; cat gpurun_out/xlane.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_sph.py tests/test_gpu_golden.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t_sph.log 2>&1; rc=$?; tail -3 gpurun_out/t_sph.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_variants.sh 4194304 30 new=tree old=abx/old/librps.so || exit $?
bash tools/prof_variants.sh 50000 100 new=tree old=abx/old/librps.so || exit $?
bash tools/prof_variants.sh 65536 100 new=tree old=abx/old/librps.so || exit $?
