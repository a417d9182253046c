#!/bin/bash
# parity + determinism suites, then tools/gpu_c1.sh with the given variants
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/c1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_determinism.py tests/test_gpu_keys.py > gpurun_out/c1/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/c1/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
exec_rc=0; tools/gpu_c1.sh "$@" || exec_rc=$?
exit $exec_rc
