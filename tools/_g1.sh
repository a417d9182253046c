mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_keys.py tests/test_gpu_stream.py tests/test_gpu_determinism.py tests/test_gpu_multirank.py tests/test_gpu_parity.py > gpurun_out/pt1.log 2>&1; rc=$?
tail -15 gpurun_out/pt1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 > gpurun_out/b1.log 2>&1; tail -c 1200 gpurun_out/b1.log
timeout -k 10 200 python bench.py --config 4 --no-cpu --no-h2d --steps 5 --warmup 2 > gpurun_out/b4.log 2>&1; tail -c 1500 gpurun_out/b4.log
