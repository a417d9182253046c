#!/bin/bash
# wide two-FE fits: dense tests (+ the 3-FE and config suites), then the headline shape at k = 10 / 14 / 20
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/wide
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dense.py \
  tests/test_gpu_dense3.py tests/test_gpu_parity.py > gpurun_out/wide/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/wide/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for k in 10 14 20; do
  timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 10 --warmup 3 --k $k > gpurun_out/wide/k$k.log 2>&1 || { tail -5 gpurun_out/wide/k$k.log; exit 1; }
  tail -1 gpurun_out/wide/k$k.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('k=$k', d['ms_per_step'], sorted([(round(v[0],3),n) for n,v in k.items()], reverse=True)[:9])"
done
for p in uhdfe_base mega_base; do
  timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 5 --warmup 2 --preset $p > gpurun_out/wide/$p.log 2>&1 || { tail -5 gpurun_out/wide/$p.log; exit 1; }
  tail -1 gpurun_out/wide/$p.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('$p', d['ms_per_step'], sorted([(round(v[0],3),n) for n,v in k.items()], reverse=True)[:9])"
done
