#!/bin/bash
# Full measurement set for profiles/: parity tests, default bench (with CPU
# baseline), rocprofv3 kernel-trace stats, PMC FETCH/WRITE passes -> traffic.
# Each GPU step has its own time limit; a fault / timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
python -m leanfe_amd.build > gpurun_out/build.log 2>&1 || { echo build failed; exit 1; }
python -c "from oracle.altproj_c import build; build()" || exit 1
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 840 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest.log; [ $rc -le 1 ] || exit $rc  # failures: still profile
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
step $? bench; tail -c 2500 gpurun_out/bench.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
  -- python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1
step $? rocprof
rm -rf gpurun_out/pmc
PASSES="fetch:FETCH_SIZE write:WRITE_SIZE" PMC_ARGS="--steps 2 --warmup 1 --no-cpu" bash tools/pmc.sh || exit $?
python tools/pmc_traffic.py gpurun_out/pmc gpurun_out/pmc_traffic.json --rows 50000000 --k 10 \
  --levels 100000,1000 --vcov HC1 > gpurun_out/pmc_traffic.log 2>&1
echo "traffic rc=$?"
