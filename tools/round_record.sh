#!/bin/bash
# End-of-round record on one GPU box: headline bench line (with the CPU baseline and the h2d
# figure), rocprofv3 kernel stats of the headline, PMC traffic of its kernels, the other configs'
# lines and the emulated 2/4/8-rank owner shards.  Everything under gpurun_out/rec/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/rec
rm -rf $out; mkdir -p $out
timeout -k 10 400 python bench.py --steps 20 --warmup 10 > $out/bench_headline.log 2>&1 || exit 1
tail -1 $out/bench_headline.log > $out/bench_headline.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv \
  -- python bench.py --steps 5 --warmup 2 --no-cpu --no-h2d > $out/prof.log 2>&1 || exit 1
echo prof ok
rm -rf gpurun_out/pmc
PASSES="fetch:FETCH_SIZE write:WRITE_SIZE" PMC_ARGS="--steps 2 --warmup 1 --no-cpu --no-h2d" bash tools/pmc.sh || exit 1
python tools/pmc_traffic.py gpurun_out/pmc $out/pmc_traffic.json --rows 50000000 --k 10 \
  --levels 100000,1000 --vcov HC1 > $out/pmc_traffic.log 2>&1
echo traffic rc=$?
: > $out/configs_bench.jsonl
for args in "--emulate-rank 0/8" "--emulate-rank 7/8" "--emulate-rank 0/4" "--emulate-rank 0/2" "--rows 6250000" \
            "--config 1" "--config 2" "--config 4 --steps 5 --warmup 2" "--config 5 --steps 5 --warmup 2"; do
  timeout -k 10 400 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $args > $out/one.log 2>&1 || { tail -5 $out/one.log; exit 1; }
  tail -1 $out/one.log >> $out/configs_bench.jsonl
  echo "$args ok"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_e8 -o run --output-format csv \
  -- python bench.py --emulate-rank 0/8 --steps 5 --warmup 2 --no-cpu --no-h2d --no-prof > $out/prof_e8.log 2>&1 || exit 1
echo done
