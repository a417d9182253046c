#!/bin/bash
# 4-bit build, Cholesky, K2 parts: the dense tests, then same-box A/Bs and a rocprof of the headline
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dense.py \
  > gpurun_out/c4/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/c4/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh LFE_DN_C4 "1 0" "--steps 20 --warmup 5" 1 || exit 1
bash tools/ab_env.sh LFE_K2_NP "2 3" "--steps 20 --warmup 5" 1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4/prof -o run \
  --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu --no-h2d > gpurun_out/c4/prof.log 2>&1 || exit 1
echo prof ok
