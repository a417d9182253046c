# A/B: batched LDS staging (new) vs per-element staging loops (old), same box; then tests
set -u
mkdir -p gpurun_out
export LFE_ALLOW_STALE=1
for r in 1 2; do
for args in "h:" "e8:--emulate-rank 0/8" "c1:--config 1"; do
  name=${args%%:*}; extra=${args#*:}
  for lib in leanfe_amd/liblfe_hip.so tools/var/old_staging.so; do
    LEANFE_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$name" "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], sys.argv[2][-16:], d["ms_per_step"], "tp", k["tp"][0], "tq", k["tq"][0], "resid", k.get("gram_resid", [0])[0])
PY
  done
done
done
unset LFE_ALLOW_STALE
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_determinism.py tests/test_gpu_parity.py tests/test_gpu_multirank.py > gpurun_out/pt19.log 2>&1; rc=$?
tail -2 gpurun_out/pt19.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/pt19.log | head -60; exit $rc; }
