# small configs: dense cross terms forced vs row layouts (the density threshold at small sizes)
set -u
mkdir -p gpurun_out
for r in 1 2; do
for args in "c1:--config 1" "c2:--config 2" "r625:--rows 6250000"; do
  name=${args%%:*}; extra=${args#*:}
  for dn in 0 1; do
    LFE_DENSE=$dn timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$name" "$dn" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], "dense" if sys.argv[2] == "1" else "rows ", d["ms_per_step"], "tp", k["tp"][0], "tq", k["tq"][0], "lsc", k.get("layout_scatter", [0])[0], "lbase", k.get("layout_base", [0])[0], d["config"].get("cross_terms"))
PY
  done
done
done
