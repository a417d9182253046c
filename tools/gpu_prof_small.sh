#!/bin/bash
# rocprofv3 kernel stats of config 1 and the HDFE panel (csv under gpurun_out/profsm/)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profsm
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profsm/c1 -o run --output-format csv \
  -- python3 bench.py --no-cpu --no-h2d --no-prof --config 1 --steps 20 --warmup 5 > gpurun_out/profsm/c1.log 2>&1 || exit 1
echo c1 ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profsm/hdfe -o run --output-format csv \
  -- python3 bench.py --no-cpu --no-h2d --no-prof --preset hdfe_base --steps 10 --warmup 3 > gpurun_out/profsm/hdfe.log 2>&1 || exit 1
echo hdfe ok
