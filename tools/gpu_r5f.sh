#!/bin/bash
# cluster sums A/B: parity (test_gpu_clusters + the clustered tests), then the clustered preset
# lines and config 4 with the sort-free one-column sums and with the sorted path (LFE_CL_FIX=0)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5f
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_clusters.py tests/test_gpu_wide.py tests/test_gpu_configs.py -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider -k "cluster or oneway or twoway or config4 or Cluster" \
  > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -le 1 ] || exit $rc
: > $out/ab.txt
for v in fix sort; do
  env_v=""; [ $v = sort ] && env_v="LFE_CL_FIX=0"
  for p in hdfe_cluster1 hdfe_cluster2 uhdfe_cluster2 mega_cluster1 mega_cluster2; do
    env $env_v timeout -k 10 300 python bench.py --no-h2d --no-cpu --steps 10 --warmup 3 --preset $p > $out/${p}_$v.log 2>&1 \
      || { tail -5 $out/${p}_$v.log; exit 1; }
    python -c "import json;d=json.loads(open('$out/${p}_$v.log').read().strip().splitlines()[-1]);k=d['kernels_ms'];print('$p $v', d['ms_per_step'], {n:k[n][0] for n in ('cluster_scatter','cluster_sort','gram_resid') if n in k})" | tee -a $out/ab.txt
  done
  env $env_v timeout -k 10 300 python bench.py --no-h2d --no-cpu --steps 3 --warmup 1 --config 4 > $out/config4_$v.log 2>&1 \
    || { tail -5 $out/config4_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('$out/config4_$v.log').read().strip().splitlines()[-1]);k=d['kernels_ms'];print('config4 $v', d['ms_per_step'], {n:k[n][0] for n in ('cluster_scatter','cluster_sort','gram_resid') if n in k})" | tee -a $out/ab.txt
done
