set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fit.py tests/test_gpu_clusters.py tests/test_gpu_multirank.py "tests/test_gpu_configs.py::test_baseline_config_vs_c_oracle[1]" "tests/test_gpu_configs.py::test_baseline_config_vs_c_oracle[3]" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_r6b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r6b.log; [ $rc -le 1 ] || exit $rc
for c in "e8:--emulate-rank 0/8" "c1:--config 1" "c3:--config 3"; do
  n=${c%%:*}; args=${c#*:}
  timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 20 --warmup 5 $args > gpurun_out/b_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/b_$n.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/b_$n.log').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['runs_ms_per_step'], d['roofline']['step']['kernel_ms'] if d.get('roofline') else '')"
done
bash tools/trace_run.sh > gpurun_out/trace.log 2>&1; echo "trace rc=$?"
