#!/bin/bash
# round-4 GPU check: dense (i8 passes) + multi-rank (owner sharding of the general sweeps), then A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dense.py \
  tests/test_gpu_multirank.py > gpurun_out/r4b_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4b_tests.log | tail -40
[ $rc -le 1 ] || exit $rc
bash tools/ab_env.sh LFE_DN8_TILED "0 1" "--steps 20 --warmup 5" 1
bash tools/ab_env.sh LFE_DN8 "1 0" "--steps 20 --warmup 5 --emulate-rank 0/8" 1
