mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_determinism.py tests/test_gpu_multirank.py tests/test_gpu_stream.py tests/test_gpu_parity.py > gpurun_out/pt2.log 2>&1; rc=$?
tail -4 gpurun_out/pt2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 > gpurun_out/b1.log 2>&1 || exit 1
head -c 300 gpurun_out/b1.log; echo
timeout -k 10 200 python bench.py --config 4 --no-cpu --no-h2d --steps 5 --warmup 2 > gpurun_out/b4.log 2>&1 || exit 1
python - <<'PY'
import json
for f in ["gpurun_out/b1.log", "gpurun_out/b4.log"]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], {k: v for k, v in d["kernels_ms"].items() if v[0] > 0.05})
PY
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr625 -o run --output-format csv -- python bench.py --rows 6250000 --steps 5 --warmup 3 --no-cpu --no-h2d --no-prof > gpurun_out/tr625.log 2>&1 || exit 1
tail -c 400 gpurun_out/tr625.log
