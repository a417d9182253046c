#!/bin/bash
# round 5 rerun: streamed factor / context tests and wide fits, the 3e9-row run, the A/B (gpu_r5c.sh)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_wide.py tests/test_gpu_stream.py -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "wide or factor or split or contexts" > gpurun_out/pytest_r5d.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r5d.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 500 python tools/oocore_run.py --rows 3000000000 --contexts 2 --chunk 50000000 --chunk2 70000000 \
  > gpurun_out/oocore_3000m.json 2> gpurun_out/oocore_3000m.err
rc=$?; echo "oocore rc=$rc"; tail -c 2500 gpurun_out/oocore_3000m.json; tail -5 gpurun_out/oocore_3000m.err
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r5c.sh
