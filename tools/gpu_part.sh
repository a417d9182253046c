#!/bin/bash
# 16-bit partition cursors: the whole GPU suite, then the shapes whose bucket count it changes
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/part
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/ > gpurun_out/part/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/part/tests.log | tail -10
[ $rc -eq 0 ] || exit $rc
for args in "--k 10" "--k 14" "--k 20" "--config 4 --steps 5 --warmup 2" "--emulate-rank 0/8"; do
  timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 10 --warmup 3 $args > gpurun_out/part/one.log 2>&1 || { tail -5 gpurun_out/part/one.log; exit 1; }
  tail -1 gpurun_out/part/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('$args', d['ms_per_step'], sorted([(round(v[0],3),n) for n,v in k.items()], reverse=True)[:6])"
done
