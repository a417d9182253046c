# dense passes: table build on 8-bit counters with returning adds (in-tree) vs 16-bit, plain adds, twice the chunks (dn_u16.so)
set -u
mkdir -p gpurun_out
for r in 1 2; do
for args in "h:" "e8:--emulate-rank 0/8"; do
  name=${args%%:*}; extra=${args#*:}
  for lib in leanfe_amd/liblfe_hip.so tools/var/dn_u16.so; do
    LFE_ALLOW_STALE=1 LEANFE_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$name" "$lib" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(sys.argv[1], sys.argv[2][-12:], d["ms_per_step"], "tp", k["tp"][0], "tq", k["tq"][0], "build", k["layout_scatter"][0])
PY
  done
done
done
