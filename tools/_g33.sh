# dense passes: two output blocks per wave (in-tree) vs one (dn_r1.so); dense tests on the new build
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_dense.py > gpurun_out/pt33.log 2>&1; rc=$?
tail -2 gpurun_out/pt33.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAILED\|assert" gpurun_out/pt33.log | head -80; exit $rc; }
for r in 1 2; do
for args in "h:" "e8:--emulate-rank 0/8"; do
  name=${args%%:*}; extra=${args#*:}
  for lib in leanfe_amd/liblfe_hip.so tools/var/dn_r1.so; do
    LFE_ALLOW_STALE=1 LEANFE_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$name" "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], sys.argv[2][-12:], d["ms_per_step"], "tp", k["tp"][0], "tq", k["tq"][0], "build", k.get("layout_scatter", [0])[0], d["config"].get("cross_terms"))
PY
  done
done
done
