set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tr
for c in "e8:--emulate-rank 0/8" "c1:--config 1" "c3:--config 3"; do
  n=${c%%:*}; args=${c#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tr/$n -o run --output-format csv -- python bench.py --no-cpu --no-h2d --no-prof --steps 6 --warmup 3 --runs 1 $args > gpurun_out/tr/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/tr/$n.log; exit 1; }
  echo "$n ok"; tail -c 300 gpurun_out/tr/$n.log
done
# host side: HIP runtime API calls beside the kernels of the 8-rank shard (no counters)
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/tr/e8api -o run --output-format csv -- python bench.py --no-cpu --no-h2d --no-prof --steps 4 --warmup 3 --runs 1 --emulate-rank 0/8 > gpurun_out/tr/e8api.log 2>&1 || { echo "e8api failed"; tail -5 gpurun_out/tr/e8api.log; exit 1; }
echo "e8api ok"
