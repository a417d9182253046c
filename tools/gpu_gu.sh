#!/bin/bash
# wide residual / design pass: GU 1 (three waves per SIMD) vs 2, tests first
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/gu
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dense.py \
  tests/test_gpu_parity.py > gpurun_out/gu/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/gu/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for k in 20 14; do
  bash tools/ab_env.sh LFE_GRAM_GU "1 2" "--steps 10 --warmup 3 --k $k" 1 || exit 1
done
