# end of round 6: full GPU suite, bench default line, config / preset lines with CPU baselines,
# rocprofv3 kernel stats, one-step traces of the 8-rank shard and configs 1 / 3
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_final.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -3 gpurun_out/bench_default.log; exit 1; }
tail -c 300 gpurun_out/bench_default.log
bash tools/measure_lines.sh > gpurun_out/measure.log 2>&1 || { tail -3 gpurun_out/measure.log; exit 1; }
echo measure ok
bash tools/trace_run.sh > gpurun_out/trace.log 2>&1 || { tail -3 gpurun_out/trace.log; exit 1; }
for n in e8 c1 c3; do python tools/trace_gaps.py gpurun_out/tr/$n/run_kernel_trace.csv > gpurun_out/trace_gaps_$n.txt; tail -1 gpurun_out/trace_gaps_$n.txt; done
