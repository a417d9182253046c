#!/bin/bash
# A/B of env variants on one box: AB_CASES="label:bench args|..." (e.g. "c4:--config 4|m1:--preset
# mega_cluster1"), AB_VARS="label:KNOB=VALUE ...|..." (engine knobs, bench --knob) (the first variant is usually "base:"), two
# repetitions; prints ms per step and the named kernel groups (AB_KERNELS, space separated)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
: > gpurun_out/ab/lines.txt
IFS='|' read -r -a cases <<< "${AB_CASES}"
IFS='|' read -r -a vars <<< "${AB_VARS}"
for rep in 1 2; do
  for cs in "${cases[@]}"; do
    cl=${cs%%:*}; args=${cs#*:}
    for vs in "${vars[@]}"; do
      vl=${vs%%:*}; ev=${vs#*:}
      f=gpurun_out/ab/${cl}_${vl}_$rep
      kn=""; for kv in $ev; do kn="$kn --knob $kv"; done  # engine knobs (the engine reads no environment)
      timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps ${AB_STEPS:-10} --warmup 3 $args $kn > $f.json 2> $f.err \
        || { tail -3 $f.err; exit 1; }
      python -c "
import json,sys
d=json.loads(open('$f.json').read().strip().splitlines()[-1]);k=d.get('kernels_ms',{})
print('$cl', '$vl', d['ms_per_step'], {n:k[n][0] for n in '${AB_KERNELS:-}'.split() if n in k})" | tee -a gpurun_out/ab/lines.txt
    done
  done
done
