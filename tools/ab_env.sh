#!/bin/bash
# Same-box A/B of an environment knob on bench lines:  tools/ab_env.sh VAR "v1 v2 ..." "bench args" [rounds]
# prints ms/step and the per-kernel ms of the dense / sweep passes for every (round, value)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
var=$1; vals=$2; args=$3; rounds=${4:-2}
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for v in $vals; do
    env $var=$v timeout -k 10 300 python bench.py --no-cpu --no-h2d $args > gpurun_out/ab_env.log 2>&1 || { tail -5 gpurun_out/ab_env.log; exit 1; }
    tail -1 gpurun_out/ab_env.log > gpurun_out/ab_env.json
    python - "$var=$v $args" <<'PY'
import json, sys
d = json.load(open("gpurun_out/ab_env.json"))
k = d["kernels_ms"]
top = sorted(k.items(), key=lambda kv: -kv[1][0])[:7]
print(sys.argv[1], d["ms_per_step"], "it", d["config"]["iterations"], " ".join(f"{n}:{v[0]:.3f}" for n, v in top), flush=True)
PY
  done
done
