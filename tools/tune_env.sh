#!/bin/bash
# time bench.py under each of several environment settings: VARIANTS="A=1 B=2;A=2" (';'-separated)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
python -m leanfe_amd.build > gpurun_out/build.log 2>&1 || exit 1
i=0
IFS=';' read -ra VS <<< "${VARIANTS:-}"
for v in "${VS[@]}"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu > gpurun_out/tune_$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "[$v] rc=$rc"; exit $rc; }
  python - "$i" "$v" <<'PY'
import json, sys
l = json.loads(open(f"gpurun_out/tune_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(f"[{sys.argv[2]}] value {l['value']} ms/step {l['ms_per_step']}", {n: v[0] for n, v in l["kernels_ms"].items() if v[0] > 0.1})
PY
done
