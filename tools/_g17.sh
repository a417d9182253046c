# A/B: K1 unit size (default rule vs one unit per wave vs 4096)
set -u
mkdir -p gpurun_out
for r in 1 2; do
for args in "h:" "e8:--emulate-rank 0/8" "c1:--config 1"; do
  name=${args%%:*}; extra=${args#*:}
  for v in def 0 4096; do
    if [ $v = def ]; then unset LFE_K1_UNIT; else export LFE_K1_UNIT=$v; fi
    timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || exit 1
    python - "$name" "$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], sys.argv[2], d["ms_per_step"], "tp", k["tp"], "iters", d["config"]["iterations"])
PY
  done
done
done
