# build counter width by bucket count: dense tests, forced-dense parity / multirank, lines
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_dense.py > gpurun_out/pt45.log 2>&1; rc=$?
tail -2 gpurun_out/pt45.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAILED\|assert" gpurun_out/pt45.log | head -80; exit $rc; }
LFE_DENSE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_multirank.py > gpurun_out/pt45a.log 2>&1; rc=$?
tail -2 gpurun_out/pt45a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAILED" gpurun_out/pt45a.log | head -80; exit $rc; }
: > gpurun_out/b45.jsonl
for args in "e8:--emulate-rank 0/8" "e8b:--emulate-rank 7/8" "e4:--emulate-rank 0/4" "e2:--emulate-rank 0/2" "h:"; do
  name=${args%%:*}; extra=${args#*:}
  timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  tail -1 gpurun_out/ab.log >> gpurun_out/b45.jsonl
  python - "$name" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], d["ms_per_step"], "tp", k["tp"][0], "tq", k["tq"][0], "build", k.get("layout_scatter", [0])[0])
PY
done
