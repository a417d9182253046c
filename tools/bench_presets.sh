#!/bin/bash
# One bench line per workload (headline + the reference's own benchmark panels, bench.PRESETS)
# into gpurun_out/presets/lines.jsonl; each run under its own time limit, stop at the first failure.
#   tools/bench_presets.sh [preset ...]      (default: all presets)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/presets
mkdir -p $out
: > $out/lines.jsonl
list=("$@")
[ ${#list[@]} -eq 0 ] && list=(hdfe_base hdfe_cluster1 hdfe_cluster2 uhdfe_base uhdfe_cluster2 mega_base mega_cluster1 mega_cluster2)
timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 > $out/headline.log 2>&1 || { tail -5 $out/headline.log; exit 1; }
tail -1 $out/headline.log >> $out/lines.jsonl
echo "headline ok"
for p in "${list[@]}"; do
  timeout -k 10 300 python bench.py --no-h2d --steps 10 --warmup 3 --preset $p > $out/$p.log 2>&1 \
    || { tail -5 $out/$p.log; exit 1; }
  tail -1 $out/$p.log >> $out/lines.jsonl
  echo "$p ok"
done
