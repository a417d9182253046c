#!/bin/bash
# the whole GPU suite (as the driver runs it at round end), then the headline A/B given as args
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/full_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/full_tests.log | tail -15
[ $rc -le 1 ] || exit $rc
[ $# -ge 3 ] && bash tools/ab_env.sh "$@"
exit $rc
