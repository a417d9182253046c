#!/bin/bash
# three-FE work: the pair-table and parity / determinism tests, then the 3-FE reference panels A/B
#   tools/gpu_d3.sh [ENV "v1 v2"]   (default A/B: LFE_SUMS_CG "1 0")
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/d3
var=${1:-LFE_SUMS_CG}
vals=${2:-"1 0"}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dense3.py \
  tests/test_gpu_parity.py tests/test_gpu_determinism.py "tests/test_gpu_multirank.py::test_emulated_owner_sharded_pair_tables" > gpurun_out/d3/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/d3/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for p in uhdfe_base mega_base; do
  for v in $vals; do
    env $var=$v timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 5 --warmup 2 --preset $p \
      > gpurun_out/d3/$p.$v.log 2>&1 || { tail -5 gpurun_out/d3/$p.$v.log; exit 1; }
    echo "$p $var=$v"; tail -1 gpurun_out/d3/$p.$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('kernels_ms'))"
  done
done
