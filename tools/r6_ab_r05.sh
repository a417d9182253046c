# same box: this engine vs the end-of-round-5 tree (tools/var/r05tree, built from e9366a6's sources),
# alternating, two repetitions per case: AB_CASES="c4:--config 4|e8:--emulate-rank 0/8|..."
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abr05
: > gpurun_out/abr05/lines.txt
IFS='|' read -r -a cases <<< "${AB_CASES:-c4:--config 4}"
for rep in 1 2; do
  for cs in "${cases[@]}"; do
    cl=${cs%%:*}; args=${cs#*:}
    for v in new r05; do
      f=$PWD/gpurun_out/abr05/${cl}_${v}_$rep.json
      if [ $v = r05 ]; then d=tools/var/r05tree; else d=.; fi
      (cd $d && timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps ${AB_STEPS:-10} --warmup 3 $args > $f 2> $f.err) || { tail -3 $f.err; exit 1; }
      python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$cl', '$v', d['ms_per_step'], d['runs_ms_per_step'])" | tee -a gpurun_out/abr05/lines.txt
    done
  done
done
