# A/B: partition chunk rows (LFE_PART_CW) on the 8-rank owner shard, 6.25M rows, config 1 and the headline
set -u
mkdir -p gpurun_out
for args in "e8:--emulate-rank 0/8" "r625:--rows 6250000" "c1:--config 1" "c2:--config 2" "h:"; do
  name=${args%%:*}; extra=${args#*:}
  for cw in auto 16384 8192 4096; do
    if [ $cw = auto ]; then unset LFE_PART_CW; else export LFE_PART_CW=$cw; fi
    timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab_${name}_${cw}.log 2>&1 || exit 1
    python - "$name" "$cw" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}_{sys.argv[2]}.log").read().strip().splitlines()[-1])
print(sys.argv[1], sys.argv[2], d["ms_per_step"], d["kernels_ms"].get("part_scatter"), d["kernels_ms"].get("group_sums"), d["kernels_ms"].get("gram_resid"))
PY
  done
done
