set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_multirank.py -k owner_shard_solves > gpurun_out/pt11.log 2>&1 || { tail -30 gpurun_out/pt11.log; exit 1; }
tail -2 gpurun_out/pt11.log
bash tools/round_record.sh
