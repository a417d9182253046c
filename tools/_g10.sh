# A/B: config 4 partition chunk rows (4096 as chosen vs 8192)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_keys.py > gpurun_out/pt10.log 2>&1 || { tail -30 gpurun_out/pt10.log; exit 1; }
tail -2 gpurun_out/pt10.log
for cw in auto 8192 auto 8192; do
  if [ $cw = auto ]; then unset LFE_PART_CW; else export LFE_PART_CW=$cw; fi
  timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 5 --warmup 2 --config 4 > gpurun_out/ab4_$cw.log 2>&1 || exit 1
  python - "$cw" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab4_{sys.argv[1]}.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], d["ms_per_step"], k.get("part_hist"), k.get("scan"), k.get("part_scatter"), k.get("group_sums"), k.get("gram_design"), k.get("gram_resid"))
PY
done
