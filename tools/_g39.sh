# small-config dense A/B, headline / 8-rank lines with the deeper build pipeline, then the config
# parity record and PMC
set -u
mkdir -p gpurun_out
bash tools/_g38.sh || exit 1
for args in "h:" "e8:--emulate-rank 0/8" "c5:--config 5 --steps 5 --warmup 2"; do
  name=${args%%:*}; extra=${args#*:}
  timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python - "$name" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], d["ms_per_step"], "tp", k["tp"][0], "tq", k["tq"][0], "build", k.get("layout_scatter", [0])[0])
PY
done
bash tools/_g37.sh
