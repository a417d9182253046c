# block-aggregated segment scatter: tests (parity, determinism, stream, configs) + config-4 A/B
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_stream.py tests/test_gpu_configs.py tests/test_gpu_multirank.py > gpurun_out/pt12.log 2>&1; rc=$?
tail -3 gpurun_out/pt12.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/pt12.log | head -60; exit $rc; }
for v in new old; do
  if [ $v = old ]; then export LFE_SEG_SCATTER_ROWS=1; else unset LFE_SEG_SCATTER_ROWS; fi
  timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 5 --warmup 2 --config 4 > gpurun_out/ab4_$v.log 2>&1 || exit 1
  python - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab4_{sys.argv[1]}.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], d["ms_per_step"], k.get("seg_build"))
PY
done
