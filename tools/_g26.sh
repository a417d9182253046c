# vectorized scans + ranged LDS histogram: GPU tests touching them, then config 4 / headline / config 1 lines
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_keys.py tests/test_gpu_multirank.py tests/test_gpu_stream.py > gpurun_out/pt26.log 2>&1; rc=$?
tail -2 gpurun_out/pt26.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/pt26.log | head -60; exit $rc; }
for args in "c4:--config 4 --steps 5 --warmup 2" "h:" "c1:--config 1"; do
  name=${args%%:*}; extra=${args#*:}
  timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/b26.log 2>&1 || { tail -5 gpurun_out/b26.log; exit 1; }
  tail -1 gpurun_out/b26.log >> gpurun_out/b26.jsonl
  python - "$name" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/b26.log").read().strip().splitlines()[-1])
print(sys.argv[1], d["ms_per_step"], {k: v[0] for k, v in d.get("kernels_ms", {}).items()})
PY
done
