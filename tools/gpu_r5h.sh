#!/bin/bash
# cluster quanta from the residual meat: parity (clusters, clustered fixtures, configs), then the
# clustered presets with meat quanta and with the statistics pass (LFE_CL_STATS=1)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5h
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_clusters.py tests/test_gpu_parity.py -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -le 1 ] || exit $rc
: > $out/ab.txt
for v in meat stats; do
  env_v=""; [ $v = stats ] && env_v="LFE_CL_STATS=1"
  for p in hdfe_cluster1 hdfe_cluster2 mega_cluster1 mega_cluster2; do
    env $env_v timeout -k 10 300 python bench.py --no-h2d --no-cpu --steps 10 --warmup 3 --preset $p > $out/${p}_$v.log 2>&1 \
      || { tail -5 $out/${p}_$v.log; exit 1; }
    python -c "import json;d=json.loads(open('$out/${p}_$v.log').read().strip().splitlines()[-1]);k=d['kernels_ms'];print('$p $v', d['ms_per_step'], {n:k[n][0] for n in ('cluster_fix','cluster_scatter','cluster_sort','gram_resid') if n in k})" | tee -a $out/ab.txt
  done
done
