# A/B: group sums with half-line loads (in-tree) vs rows 4kq..4kq+3 per lane (sums_old.so); then
# the parity / determinism tests of the new build
set -u
mkdir -p gpurun_out
for r in 1 2 3; do
for args in "h:" "e8:--emulate-rank 0/8"; do
  name=${args%%:*}; extra=${args#*:}
  for lib in leanfe_amd/liblfe_hip.so tools/var/sums_old.so; do
    LFE_ALLOW_STALE=1 LEANFE_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$name" "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], sys.argv[2][-20:], d["ms_per_step"], "sums", k["group_sums"][0], "part", k["part_scatter"][0])
PY
  done
done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_determinism.py tests/test_gpu_parity.py > gpurun_out/pt24.log 2>&1; rc=$?
tail -2 gpurun_out/pt24.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/pt24.log | head -60; exit $rc; }
