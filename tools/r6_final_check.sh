# full GPU suite on the final library, then kernel + runtime traces of the 8-rank shard and configs
# 1 and 3 (trace_gaps summaries for profiles/)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_final.log; [ $rc -le 1 ] || exit $rc
rm -rf gpurun_out/tr
bash tools/trace_run.sh > gpurun_out/trace.log 2>&1; echo "trace rc=$?"
for n in e8 c1 c3; do python tools/trace_gaps.py gpurun_out/tr/$n/run_kernel_trace.csv > gpurun_out/trace_gaps_$n.txt; tail -1 gpurun_out/trace_gaps_$n.txt; done
