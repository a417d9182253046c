# probe: the engine's RCCL path with 2 ranks on one GPU (owner shards, then row shards)
set -u
mkdir -p gpurun_out
export LEANFE_BENCH_DEVICE=0 NCCL_DEBUG=WARN
timeout -k 10 180 python bench.py --gpus 2 --rows 2000000 --steps 3 --warmup 1 --no-cpu --no-h2d --verbose > gpurun_out/r2o.log 2>&1; echo "owner rc=$?"; tail -c 1500 gpurun_out/r2o.log
