# wide tests + the multi-row cluster test, MEGA_CLUSTER2 / config 4 A/B of the multi-row corrections,
# then the 1e9-row wide fit
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_wide.py \
  "tests/test_gpu_clusters.py::test_mostly_singleton_intersection_multi_row_corrections" > gpurun_out/r6_run1_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6_run1_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "fused:" "gather:LFE_CL_MULTI_GATHER=1"; do
  n=${v%%:*}; kv=${v#*:}; ka=""; [ -n "$kv" ] && ka="--knob $kv"
  for p in "--preset mega_cluster2" "--config 4"; do
    timeout -k 10 200 python bench.py --no-cpu --no-h2d --steps 6 --warmup 2 $p $ka > gpurun_out/r6_ab_tmp.log 2>&1 || { tail -5 gpurun_out/r6_ab_tmp.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/r6_ab_tmp.log').read().strip().splitlines()[-1]); print('$n', '$p', d['ms_per_step'], d['runs_ms_per_step'])"
  done
done
timeout -k 10 600 python -u tools/wide_oocore_run.py --rows 1000000000 --k 100 --chunk 20000000 --chunk2 32000000 \
  > gpurun_out/wide_1e9.json 2> gpurun_out/wide_1e9.err
echo "wide rc=$?"; tail -c 1500 gpurun_out/wide_1e9.json
