#!/bin/bash
# round 5: A/B on one box - group-sums form, partition geometry, K1 digit source - on the headline,
# config 1 and the 8-rank owner shard
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/ab_r5c.txt
run() {  # label, bench args (quoted), env...
  local label=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $args > gpurun_out/ab_$label.json 2>gpurun_out/ab_$label.err || { tail -3 gpurun_out/ab_$label.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$label.json'));k=d['kernels_ms'];g=lambda n:k.get(n,[0])[0];print('$label', d['ms_per_step'], 'part', g('part_scatter'), 'sums', g('group_sums'), 'resid', g('gram_resid'), 'tp', g('tp'))" | tee -a gpurun_out/ab_r5c.txt
}
for rep in 1 2; do
  run base$rep ""
  run mfma$rep "" LFE_SUMS_ROWS=0
  run g36_$rep "" LFE_PART_GEOM=512,36
  run g32_$rep "" LFE_PART_GEOM=512,32
  run k1own$rep "" LFE_DN8_PRE=0
  run c1_$rep "--config 1"
  run c1own$rep "--config 1" LFE_DN8_PRE=0
  run e8_$rep "--emulate-rank 0/8"
  run e8own$rep "--emulate-rank 0/8" LFE_DN8_PRE=0
done
