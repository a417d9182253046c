#!/bin/bash
# small-config A/B (config $CFG, default 1): default vs env variants given as args ("NAME=V NAME2=V2" each)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/c1
cfg=${CFG:-1}
for v in "" "$@"; do
  env $v timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 --config $cfg ${EXTRA:-} > gpurun_out/c1/run.log 2>&1 || { tail -5 gpurun_out/c1/run.log; exit 1; }
  tail -1 gpurun_out/c1/run.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('[$v]', d['ms_per_step'], d['runs_ms_per_step'], sorted([(round(v[0],3),n) for n,v in k.items()], reverse=True)[:12])"
done
