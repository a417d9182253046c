# kernel stats + traces: config 4 (where its scan / count time goes) and config 1 (fixed cost)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p4 -o run --output-format csv \
  -- python bench.py --config 4 --steps 2 --warmup 1 --no-cpu --no-h2d --no-prof > gpurun_out/p4.log 2>&1 || { tail -5 gpurun_out/p4.log; exit 1; }
echo p4 ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p1 -o run --output-format csv \
  -- python bench.py --config 1 --steps 5 --warmup 2 --no-cpu --no-h2d --no-prof > gpurun_out/p1.log 2>&1 || { tail -5 gpurun_out/p1.log; exit 1; }
echo p1 ok
