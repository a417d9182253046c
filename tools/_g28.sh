# K2 rows-per-workgroup minimum (LFE_K2_MINROWS) at the 8-rank owner shard, config 1 and the headline
set -u
mkdir -p gpurun_out
for r in 1 2; do
for args in "e8:--emulate-rank 0/8" "c1:--config 1" "c2:--config 2" "h:"; do
  name=${args%%:*}; extra=${args#*:}
  for mr in 16384 8192 4096; do
    LFE_K2_MINROWS=$mr timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$name" "$mr" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], sys.argv[2], d["ms_per_step"], "tq", k["tq"][0], "tp", k["tp"][0])
PY
  done
done
done
