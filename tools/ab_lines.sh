#!/bin/bash
# A/B on one box: the headline, config 1 and the 8-rank owner shard, with optional env overrides
# (AB_ENV="NAME=VALUE ..." for the variant runs), two repetitions each
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/ab_lines.txt
run() {  # label, bench args (quoted), env...
  local label=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $args > gpurun_out/ab_$label.json 2>gpurun_out/ab_$label.err || { tail -3 gpurun_out/ab_$label.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$label.json'));k=d['kernels_ms'];g=lambda n:k.get(n,[0])[0];print('$label', d['ms_per_step'], 'part', g('part_scatter'), 'sums', g('group_sums'), 'resid', g('gram_resid'), 'tp', g('tp'))" | tee -a gpurun_out/ab_lines.txt
}
for rep in 1 2; do
  run base$rep ""
  run c1_$rep "--config 1"
  run e8_$rep "--emulate-rank 0/8"
  if [ -n "${AB_ENV:-}" ]; then
    run var$rep "" $AB_ENV
    run c1var$rep "--config 1" $AB_ENV
    run e8var$rep "--emulate-rank 0/8" $AB_ENV
  fi
done
