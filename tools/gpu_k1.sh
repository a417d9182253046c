#!/bin/bash
# dense passes / tables-Gram changes: dense + multirank + config tests, then a rocprof of the headline
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/k1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dense.py \
  tests/test_gpu_multirank.py "tests/test_gpu_configs.py::test_baseline_config_vs_c_oracle" > gpurun_out/k1/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/k1/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 > gpurun_out/k1/bench.log 2>&1 || exit 1
tail -1 gpurun_out/k1/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['runs_ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k1/prof -o run \
  --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu --no-h2d > gpurun_out/k1/prof.log 2>&1 || exit 1
echo prof ok
