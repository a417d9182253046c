#!/bin/bash
# K2-formed alpha_P + resident-aware K2 split: parity suites, per-workgroup timing, configs 1 / 2 /
# HDFE A/B against LFE_K2FIN=0
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/k2f
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_determinism.py tests/test_gpu_multirank.py tests/test_gpu_keys.py tests/test_gpu_dense.py \
  tests/test_gpu_configs.py -k "not config5" > gpurun_out/k2f/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/k2f/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
tools/gpu_swt.sh || exit 1
for a in "--config 1" "--config 2" "--preset hdfe_base"; do
  for v in "" "LFE_K2FIN=0"; do
    env $v timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $a > gpurun_out/k2f/run.log 2>&1 || { tail -5 gpurun_out/k2f/run.log; exit 1; }
    tail -1 gpurun_out/k2f/run.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('$a [$v]', d['ms_per_step'], d['runs_ms_per_step'], sorted([(round(v[0],3),n) for n,v in k.items()], reverse=True)[:5])"
  done
done
