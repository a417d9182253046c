#!/bin/bash
# Tuning sweep on one box: bench.py once per value of an engine tuning knob (bench --knob).
#   VAR=SOME_ENV VALUES="1 2 4" KEYS="tq,tp" bash tools/tune_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VALUES}; do
  timeout -k 10 120 python bench.py --no-cpu --steps ${STEPS:-10} --warmup 5 --knob ${VAR}=${v} > gpurun_out/tune_${v}.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "${VAR}=${v} rc=$rc"; tail -3 gpurun_out/tune_${v}.log; exit $rc; }
  python - "$v" "${KEYS:-}" <<'PY'
import json, sys
v, keys = sys.argv[1], [k for k in sys.argv[2].split(",") if k]
d = json.loads([l for l in open(f"gpurun_out/tune_{v}.log") if l.startswith("{")][-1])
ks = d["kernels_ms"]
print(f"{v:>8}: {d['ms_per_step']:.3f} ms/step  " + "  ".join(f"{k}={ks[k][0]:.4f}" for k in keys if k in ks))
PY
done
