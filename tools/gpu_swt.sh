#!/bin/bash
# per-workgroup wall clock of the row-layout sweeps' K1 / K2 (LFE_SWEEP_TIMING) on configs 1, 2 and the HDFE panel
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/swt
for a in "--config 1" "--config 2" "--preset hdfe_base"; do
  LFE_SWEEP_TIMING=1 timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 1 --warmup 1 --runs 1 --no-prof $a > gpurun_out/swt/run.log 2>&1 || { tail -5 gpurun_out/swt/run.log; exit 1; }
  echo "$a"; grep -E "^K[12] " gpurun_out/swt/run.log | tail -2
done
