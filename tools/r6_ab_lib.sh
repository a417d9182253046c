# same-box A/B of the in-tree library against a variant build (LEANFE_HIP_LIB), two repetitions:
#   AB_LIB=tools/var/x.so AB_CASES="c4:--config 4|..." AB_KERNELS="cross" bash tools/r6_ab_lib.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ablib
: > gpurun_out/ablib/lines.txt
IFS='|' read -r -a cases <<< "${AB_CASES}"
for rep in 1 2; do
  for cs in "${cases[@]}"; do
    cl=${cs%%:*}; args=${cs#*:}
    for v in new old; do
      f=gpurun_out/ablib/${cl}_${v}_$rep
      if [ $v = old ]; then lib="$AB_LIB"; else lib=""; fi
      LEANFE_HIP_LIB=$lib LFE_ALLOW_STALE=$([ $v = old ] && echo 1 || echo 0) timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps ${AB_STEPS:-6} --warmup 2 $args > $f.json 2> $f.err \
        || { tail -3 $f.err; exit 1; }
      python -c "
import json
d=json.loads(open('$f.json').read().strip().splitlines()[-1]);k=d.get('kernels_ms',{})
print('$cl', '$v', d['ms_per_step'], {n:(k[n][0], round(k[n][0]/k[n][1],4)) for n in '${AB_KERNELS:-}'.split() if n in k})" | tee -a gpurun_out/ablib/lines.txt
    done
  done
done
