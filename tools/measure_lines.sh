#!/bin/bash
# Measurement set beside round_profile.sh: preset lines (with CPU baselines), config lines 1-5 and
# the 8-rank owner shard, then rocprofv3 kernel stats of config 1, config 4, the shard and the
# clustered presets (profiles/rNN/presets_bench.jsonl, configs_bench.jsonl, *_kernel_stats.csv).
# Any failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/lines
mkdir -p $out
: > $out/configs.jsonl
bash tools/bench_presets.sh || exit $?
for c in 1 2 3 4 5; do
  # every config line with its CPU baseline (config 5: the first 5e7 rows of its 5e8-row panel)
  timeout -k 10 300 python bench.py --no-h2d --cpu-rows 50000000 --steps 10 --warmup 3 --config $c > $out/config$c.log 2>&1 \
    || { tail -5 $out/config$c.log; exit 1; }
  tail -1 $out/config$c.log >> $out/configs.jsonl; echo "config $c ok"
done
timeout -k 10 300 python bench.py --no-h2d --no-cpu --steps 20 --warmup 5 --emulate-rank 0/8 > $out/e8.log 2>&1 \
  || { tail -5 $out/e8.log; exit 1; }
tail -1 $out/e8.log >> $out/configs.jsonl; echo "e8 ok"
export TMPDIR=/tmp
prof() {  # name, bench args
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$name -o run --output-format csv \
    -- python bench.py --no-h2d --no-cpu "$@" > $out/prof_$name.log 2>&1 || { tail -5 $out/prof_$name.log; exit 1; }
  echo "prof $name ok"
}
prof config1 --steps 20 --warmup 3 --config 1
prof e8 --steps 10 --warmup 3 --emulate-rank 0/8
prof config4 --steps 2 --warmup 1 --config 4
prof hdfe_cluster2 --steps 5 --warmup 2 --preset hdfe_cluster2
prof mega_cluster2 --steps 3 --warmup 1 --preset mega_cluster2
