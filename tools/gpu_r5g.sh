#!/bin/bash
# sort-free one-column cluster sums: parity, clustered presets (fix form), kernel stats of two of them
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5g
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_clusters.py -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -le 1 ] || exit $rc
: > $out/ab.txt
for p in hdfe_cluster1 hdfe_cluster2 uhdfe_cluster2 mega_cluster1 mega_cluster2; do
  timeout -k 10 300 python bench.py --no-h2d --no-cpu --steps 10 --warmup 3 --preset $p > $out/$p.log 2>&1 \
    || { tail -5 $out/$p.log; exit 1; }
  python -c "import json;d=json.loads(open('$out/$p.log').read().strip().splitlines()[-1]);k=d['kernels_ms'];print('$p', d['ms_per_step'], {n:k[n][0] for n in ('cluster_scatter','cluster_sort','gram_resid') if n in k})" | tee -a $out/ab.txt
done
export TMPDIR=/tmp
for p in hdfe_cluster1 mega_cluster1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$p -o run --output-format csv \
    -- python bench.py --no-h2d --no-cpu --steps 5 --warmup 2 --preset $p > $out/prof_$p.log 2>&1 || { tail -5 $out/prof_$p.log; exit 1; }
done
