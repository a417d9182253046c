# round-3 session 2: baseline timings at HEAD (headline, 8-rank owner shard, config 1, config 4) + traces
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 > gpurun_out/h.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 --emulate-rank 0/8 > gpurun_out/e8.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 --rows 6250000 > gpurun_out/r625.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 --config 1 > gpurun_out/c1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 5 --warmup 2 --config 4 > gpurun_out/c4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tre8 -o run --output-format csv -- python bench.py --emulate-rank 0/8 --steps 5 --warmup 3 --no-cpu --no-h2d --no-prof > gpurun_out/tre8.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trc4 -o run --output-format csv -- python bench.py --config 4 --steps 2 --warmup 1 --no-cpu --no-h2d --no-prof > gpurun_out/trc4.log 2>&1 || exit 1
python - <<'PY'
import json
for f in ["h", "e8", "r625", "c1", "c4"]:
    d = json.loads(open(f"gpurun_out/{f}.log").read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], d["config"]["iterations"], {k: v for k, v in d["kernels_ms"].items() if v[0] > 0.02})
PY
