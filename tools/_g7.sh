# kernel trace of the emulated 8-rank owner shard and of config 1
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tre8 -o run --output-format csv -- python bench.py --emulate-rank 0/8 --steps 5 --warmup 3 --no-cpu --no-h2d --no-prof > gpurun_out/tre8.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trc1 -o run --output-format csv -- python bench.py --config 1 --steps 5 --warmup 3 --no-cpu --no-h2d --no-prof > gpurun_out/trc1.log 2>&1 || exit 1
