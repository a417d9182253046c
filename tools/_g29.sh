# column-split LDS sums for config 4's third FE: parity / determinism / stream / multirank tests,
# config 4 at full size vs the C oracle, then the config 4 bench line
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_stream.py tests/test_gpu_multirank.py > gpurun_out/pt29.log 2>&1; rc=$?
tail -2 gpurun_out/pt29.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/pt29.log | head -60; exit $rc; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -p no:cacheprovider "tests/test_gpu_configs.py::test_baseline_config_vs_c_oracle[4]" > gpurun_out/pt29c.log 2>&1; rc=$?
tail -2 gpurun_out/pt29c.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/pt29c.log | head -60; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu --no-h2d --config 4 --steps 5 --warmup 2 > gpurun_out/b29.log 2>&1 || { tail -5 gpurun_out/b29.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/b29.log").read().strip().splitlines()[-1])
print("c4", d["ms_per_step"], {k: v[0] for k, v in d.get("kernels_ms", {}).items()})
PY
