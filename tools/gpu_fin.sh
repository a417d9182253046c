#!/bin/bash
# validation after the K2 split change: parity / determinism / configs suites, then the bench lines
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/fin
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_determinism.py tests/test_gpu_multirank.py tests/test_gpu_keys.py tests/test_gpu_dense.py \
  tests/test_gpu_configs.py -k "not config5" > gpurun_out/fin/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/fin/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/fin/lines.jsonl
for a in "--config 1" "--config 2" "--preset hdfe_base" "--emulate-rank 0/8" "--config 3"; do
  timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $a > gpurun_out/fin/run.log 2>&1 || { tail -5 gpurun_out/fin/run.log; exit 1; }
  tail -1 gpurun_out/fin/run.log >> gpurun_out/fin/lines.jsonl
  tail -1 gpurun_out/fin/run.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['ms_per_step'], d['runs_ms_per_step'])"
done
