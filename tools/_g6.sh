# K1 empty-segment skip + K2 over non-empty buckets: GPU tests (parity, multirank, determinism) + benches
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_determinism.py > gpurun_out/pt6.log 2>&1; rc=$?
tail -5 gpurun_out/pt6.log
[ $rc -eq 0 ] || exit $rc
for args in "h:" "e8:--emulate-rank 0/8" "e87:--emulate-rank 7/8" "e4:--emulate-rank 0/4" "r625:--rows 6250000" "c1:--config 1"; do
  name=${args%%:*}; extra=${args#*:}
  timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/$name.log 2>&1 || exit 1
done
python - <<'PY'
import json
for f in ["h", "e8", "e87", "e4", "r625", "c1"]:
    d = json.loads(open(f"gpurun_out/{f}.log").read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], d["config"]["iterations"], d["config"]["rows_rank0"], {k: v for k, v in d["kernels_ms"].items() if v[0] > 0.02})
PY
