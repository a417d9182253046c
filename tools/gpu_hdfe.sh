#!/bin/bash
# two-FE row kernels at G_Q = 2000 (the HDFE panels): parity suites, then the hdfe presets + headline
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/hdfe
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_dense.py tests/test_gpu_configs.py -k "not config5" > gpurun_out/hdfe/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/hdfe/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for p in headline hdfe_base hdfe_cluster1 hdfe_cluster2; do
  arg="--preset $p"; [ $p = headline ] && arg=""
  timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 10 --warmup 3 $arg > gpurun_out/hdfe/$p.log 2>&1 || { tail -5 gpurun_out/hdfe/$p.log; exit 1; }
  tail -1 gpurun_out/hdfe/$p.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('$p', d['ms_per_step'], sorted([(round(v[0],3),n) for n,v in k.items()], reverse=True)[:9])"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hdfe/prof_c1 -o c1 -- python3 bench.py --no-cpu --no-h2d --no-prof --config 1 --steps 20 --warmup 5 > gpurun_out/hdfe/c1_prof.log 2>&1 || { tail -5 gpurun_out/hdfe/c1_prof.log; exit 1; }
echo c1 prof ok
