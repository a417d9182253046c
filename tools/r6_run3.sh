# quick parity subset, then same-box A/B of where the bucket starts are read (main stream before the
# scatter vs side stream) with the work items copied by a kernel from mapped staging
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_fit.py \
  tests/test_gpu_knobs.py "tests/test_gpu_configs.py::test_baseline_config_vs_c_oracle[1]" tests/test_gpu_multirank.py \
  > gpurun_out/r6_run3_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6_run3_tests.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=20 AB_CASES="e8:--emulate-rank 0/8|c1:--config 1|c2:--config 2|c3:--config 3" \
  AB_VARS="dflt:|main:LFE_BSTART_MAIN_ROWS=1000000000|side:LFE_BSTART_MAIN_ROWS=0" bash tools/ab_env.sh || exit $?
cp gpurun_out/ab/lines.txt gpurun_out/ab_bstart.txt
