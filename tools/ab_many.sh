#!/bin/bash
# Same-box A/B of several engine builds: LIBS="a.so b.so" KEYS="part_scatter" ROUNDS=2 bash tools/ab_many.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS}; do
    LFE_ALLOW_STALE=1 LEANFE_HIP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu --no-h2d --steps ${STEPS:-10} --warmup 5 ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -3 gpurun_out/ab.log; exit $rc; }
    python - "$lib" "${KEYS:-}" <<'PY'
import json, sys
lib, keys = sys.argv[1], [k for k in sys.argv[2].split(",") if k]
d = json.loads([l for l in open("gpurun_out/ab.log") if l.startswith("{")][-1])
ks = d["kernels_ms"]
st = d.get("roofline", {}).get("step", {})
print(f"{lib:>28}: {d['ms_per_step']:.3f} ms/step  kern={st.get('kernel_ms', 0):.3f} gap={st.get('host_gap_ms', 0):.3f}  " + "  ".join(f"{k}={ks[k][0]:.4f}" for k in keys if k in ks), flush=True)
if len(keys) == 1 and keys[0] == "all":
    print("   " + " ".join(f"{k}={v[0]:.4f}/{v[1]}" for k, v in ks.items()), flush=True)
PY
  done
done
