#!/bin/bash
# kernel stats of HDFE_CLUSTER1 with meat quanta and with the statistics pass
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5i
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_meat -o run --output-format csv \
  -- python bench.py --no-h2d --no-cpu --steps 10 --warmup 3 --preset hdfe_cluster1 > $out/prof_meat.log 2>&1 || exit 1
LFE_CL_STATS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_stats -o run --output-format csv \
  -- python bench.py --no-h2d --no-cpu --steps 10 --warmup 3 --preset hdfe_cluster1 > $out/prof_stats.log 2>&1 || exit 1
echo ok
