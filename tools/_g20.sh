# HEAD check at round-3 re-entry: full GPU suite, then headline / 8-rank shard / config 1 bench lines
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt20.log 2>&1; rc=$?
tail -3 gpurun_out/pt20.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/pt20.log | head -80; exit $rc; }
for args in "h:" "e8:--emulate-rank 0/8" "c1:--config 1" "c4:--config 4 --steps 5 --warmup 2"; do
  name=${args%%:*}; extra=${args#*:}
  timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $extra > gpurun_out/b20.log 2>&1 || { tail -5 gpurun_out/b20.log; exit 1; }
  tail -1 gpurun_out/b20.log >> gpurun_out/b20.jsonl
  python - "$name" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/b20.log").read().strip().splitlines()[-1])
print(sys.argv[1], d["ms_per_step"], {k: v[0] for k, v in d.get("kernels_ms", {}).items()})
PY
done
