# dense count-table cross terms: tests forced dense (LFE_DENSE=1), then default; bench lines dense vs layouts
set -u
mkdir -p gpurun_out
LFE_DENSE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_multirank.py > gpurun_out/pt30a.log 2>&1; rc=$?
tail -2 gpurun_out/pt30a.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAILED" gpurun_out/pt30a.log | head -80; exit $rc; }
for r in 1 2; do
for args in "h:" "e8:--emulate-rank 0/8" "c2:--config 2" "c1:--config 1"; do
  name=${args%%:*}; extra=${args#*:}
  for dn in 0 1; do
    LFE_DENSE=$dn timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$name" "$dn" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], "dense" if sys.argv[2] == "1" else "rows ", d["ms_per_step"], "tp", k["tp"][0], "tq", k["tq"][0], "lsc", k.get("layout_scatter", [0])[0], "lbase", k.get("layout_base", [0])[0])
PY
  done
done
done
