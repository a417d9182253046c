mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -x -q -s --timeout 1000 --timeout-method thread -p no:cacheprovider tests/test_gpu_configs.py > gpurun_out/cfg.log 2>&1; rc=$?
grep '^{' gpurun_out/cfg.log > gpurun_out/cfg.jsonl; tail -5 gpurun_out/cfg.log
exit $rc
