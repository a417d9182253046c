#!/bin/bash
# round 5: streamed factor terms, context split, 3e9-row out-of-core fit on one GPU
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_stream.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "factor or split or contexts" > gpurun_out/pytest_r5a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r5a.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/oocore_run.py --rows 3000000000 --contexts 2 --chunk 50000000 --chunk2 70000000 \
  > gpurun_out/oocore_3000m.json 2> gpurun_out/oocore_3000m.err
rc=$?; echo "oocore rc=$rc"; tail -c 2500 gpurun_out/oocore_3000m.json; tail -5 gpurun_out/oocore_3000m.err
