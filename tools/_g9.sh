# cluster columns moved by the partition + parallel k_cross_quanta: GPU tests incl. full-size configs, config 4 bench
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_determinism.py tests/test_gpu_configs.py > gpurun_out/pt9.log 2>&1; rc=$?
tail -4 gpurun_out/pt9.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 5 --warmup 2 --config 4 > gpurun_out/c4.log 2>&1 || exit 1
python - <<'PY'
import json
d = json.loads(open("gpurun_out/c4.log").read().strip().splitlines()[-1])
print("c4", d["ms_per_step"], d["config"]["iterations"], {k: v for k, v in d["kernels_ms"].items() if v[0] > 0.05})
PY
