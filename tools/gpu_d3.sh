#!/bin/bash
# pair-table sweeps (lfe_dense3.hip): their tests, then the 3-FE reference panels with and without them
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/d3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dense3.py \
  > gpurun_out/d3/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/d3/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for p in uhdfe_base mega_base; do
  for d in 1 0; do
    LFE_DENSE=$([ $d = 0 ] && echo 0 || echo auto) timeout -k 10 300 python bench.py --no-cpu --no-h2d \
      --steps 5 --warmup 2 --preset $p > gpurun_out/d3/$p.$d.log 2>&1 || { tail -5 gpurun_out/d3/$p.$d.log; exit 1; }
    echo "$p dense=$d"; tail -1 gpurun_out/d3/$p.$d.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('kernels_ms'))" 2>/dev/null || tail -2 gpurun_out/d3/$p.$d.log
  done
done
