#!/bin/bash
# round 5: A/B of the group-sums form and the partition geometry on the headline (same box)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/ab_r5c.txt
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 > gpurun_out/ab_$label.json 2>gpurun_out/ab_$label.err || { tail -3 gpurun_out/ab_$label.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$label.json'));k=d['kernels_ms'];print('$label', d['ms_per_step'], 'part', k['part_scatter'][0], 'sums', k['group_sums'][0], 'resid', k['gram_resid'][0])" | tee -a gpurun_out/ab_r5c.txt
}
for rep in 1 2; do
  run base$rep LFE_SUMS_ROWS=1
  run mfma$rep LFE_SUMS_ROWS=0
  run g36_$rep LFE_PART_GEOM=512,36
  run g32_$rep LFE_PART_GEOM=512,32
done
