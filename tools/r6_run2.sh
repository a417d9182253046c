# multi-row cluster test, then same-box A/Bs: the multi-row corrections (MEGA_CLUSTER2, config 4) and
# the host messages (8-rank shard, configs 1 and 3)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread \
  "tests/test_gpu_clusters.py::test_mostly_singleton_intersection_multi_row_corrections" > gpurun_out/r6_run2_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6_run2_tests.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=6 AB_CASES="m2:--preset mega_cluster2|c4:--config 4" AB_VARS="direct:|gather:LFE_CL_MULTI_GATHER=1" \
  AB_KERNELS="cluster_scatter gram_table" bash tools/ab_env.sh || exit $?
cp gpurun_out/ab/lines.txt gpurun_out/ab_multi.txt
AB_STEPS=20 AB_CASES="e8:--emulate-rank 0/8|c1:--config 1|c3:--config 3" AB_VARS="msg:|nomsg:LFE_HOST_MSG=0" bash tools/ab_env.sh || exit $?
cp gpurun_out/ab/lines.txt gpurun_out/ab_hostmsg.txt
