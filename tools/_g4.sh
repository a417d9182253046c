set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
  -- python bench.py --steps 5 --warmup 2 --no-cpu --no-h2d > gpurun_out/prof.log 2>&1 || exit 1
echo prof ok
rm -rf gpurun_out/pmc
PASSES="fetch:FETCH_SIZE write:WRITE_SIZE" PMC_ARGS="--steps 2 --warmup 1 --no-cpu --no-h2d" bash tools/pmc.sh || exit 1
python tools/pmc_traffic.py gpurun_out/pmc gpurun_out/pmc_traffic.json --rows 50000000 --k 10 \
  --levels 100000,1000 --vcov HC1 > gpurun_out/pmc_traffic.log 2>&1
echo traffic rc=$?
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/bench_full.log 2>&1
echo bench rc=$?; tail -c 600 gpurun_out/bench_full.log
