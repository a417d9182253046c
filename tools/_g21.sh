# A/B (diagnostic): partition writes into 64-row tiles of all p columns vs column-major bucket runs
set -u
mkdir -p gpurun_out
export LFE_ALLOW_STALE=1
for r in 1 2 3; do
  for lib in leanfe_amd/liblfe_hip.so tools/var/tile_diag.so; do
    LEANFE_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1][-22:], d["ms_per_step"], "part", k["part_scatter"][0], "sums", k["group_sums"][0], "resid", k.get("gram_resid", [0])[0])
PY
  done
done
