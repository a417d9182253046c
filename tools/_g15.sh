# sweep LDS pitch A/B (LFE_SWEEP_PITCH=0: packed rows) + parity/determinism tests
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_multirank.py > gpurun_out/pt15.log 2>&1; rc=$?
tail -2 gpurun_out/pt15.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/pt15.log | head -60; exit $rc; }
for r in 1 2; do
for args in "h:" "e8:--emulate-rank 0/8" "c1:--config 1"; do
  name=${args%%:*}; extra=${args#*:}
  for v in new old; do
    if [ $v = old ]; then export LFE_SWEEP_PITCH=0; else unset LFE_SWEEP_PITCH; fi
    timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || exit 1
    python - "$name" "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], sys.argv[2], d["ms_per_step"], "tp", k["tp"], "tq", k["tq"])
PY
  done
done
done
