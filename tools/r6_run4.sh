# parity subset for the small-upload change, then same-box A/B (kernel copy vs SDMA) on the paths
# that upload (three FEs, clusters)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 250 --timeout-method thread tests/test_gpu_clusters.py \
  tests/test_gpu_seg_build.py "tests/test_gpu_configs.py::test_baseline_config_vs_c_oracle[4]" tests/test_gpu_knobs.py \
  > gpurun_out/r6_run4_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r6_run4_tests.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=6 AB_CASES="c4:--config 4|h2:--preset hdfe_cluster2|h1:--preset hdfe_cluster1|m2:--preset mega_cluster2|u2:--preset uhdfe_cluster2" \
  AB_VARS="kern:|sdma:LFE_H2D_SDMA=1" bash tools/ab_env.sh || exit $?
cp gpurun_out/ab/lines.txt gpurun_out/ab_h2d.txt
