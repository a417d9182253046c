#!/bin/bash
# GPU round: build, parity tests, headline bench, rocprof kernel trace.  Every GPU
# step has its own time limit; a crash/timeout (rc >= 124 or signal) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
python -m leanfe_amd.build > gpurun_out/build.log 2>&1 || { echo build failed; exit 1; }
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [ "${RUN_TESTS:-1}" = 1 ]; then
  eval "set -- ${PYTEST_ARGS:-}"  # shell-quoted extra arguments, e.g. PYTEST_ARGS="-k 'a or b'"
  timeout -k 10 ${TEST_TIMEOUT:-500} python -m pytest tests -m gpu -q -x -p no:cacheprovider "$@" > gpurun_out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest.log
  ok $rc || exit $rc
fi
if [ "${RUN_BENCH:-1}" = 1 ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${RUN_PROF:-0}" = 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py ${PROF_ARGS:---steps 3 --warmup 1 --no-cpu} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -5 gpurun_out/prof.log
fi
