#!/bin/bash
# time bench.py under each LFE_GRAM_GU / LFE_SUMS_GU setting (tuning helper)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
python -m leanfe_amd.build > gpurun_out/build.log 2>&1 || exit 1
for gu in ${GUS:-1 2 4}; do
  LFE_GRAM_GU=$gu LFE_SUMS_GU=$gu timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/tune_gu$gu.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "gu=$gu rc=$rc"; exit $rc; }
  python - "$gu" <<'PY'
import json, sys
l = json.loads(open(f"gpurun_out/tune_gu{sys.argv[1]}.log").read().strip().splitlines()[-1])
k = l["kernels_ms"]
print("gu", sys.argv[1], "value", l["value"], {n: k[n][0] for n in ("group_sums", "gram_design", "gram_resid") if n in k})
PY
done
