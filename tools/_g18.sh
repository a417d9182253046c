set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_determinism.py tests/test_gpu_parity.py tests/test_gpu_multirank.py > gpurun_out/pt18.log 2>&1; rc=$?
tail -2 gpurun_out/pt18.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/pt18.log | head -60; exit $rc; }
for args in "h:" "e8:--emulate-rank 0/8" "c1:--config 1" "c2:--config 2"; do
  name=${args%%:*}; extra=${args#*:}
  timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || exit 1
  python - "$name" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], d["ms_per_step"], "tp", k["tp"], "tq", k["tq"])
PY
done
