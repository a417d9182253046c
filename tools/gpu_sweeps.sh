#!/bin/bash
# k_sweeps per-phase wall clock (LFE_SWEEP_TIMING) on config 1 and the HDFE shape
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sw
LFE_PERSIST=1 LFE_SWEEP_TIMING=1 timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 2 --warmup 1 --runs 1 --no-prof --config 1 > gpurun_out/sw/c1.log 2>&1 || { tail -5 gpurun_out/sw/c1.log; exit 1; }
grep "k_sweeps timing" gpurun_out/sw/c1.log | tail -2
