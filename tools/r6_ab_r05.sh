# same-box: config 4 on the in-tree engine vs the end-of-round-5 tree (tools/var/r05tree)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abr05
for rep in 1 2; do
  for v in new r05; do
    f=$PWD/gpurun_out/abr05/${v}_$rep.json
    if [ $v = r05 ]; then d=tools/var/r05tree; else d=.; fi
    (cd $d && timeout -k 10 300 python bench.py --no-cpu --no-h2d --steps 4 --warmup 2 --config 4 > $f 2> $f.err) || { tail -3 $f.err; exit 1; }
    python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]);k=d.get('kernels_ms',{})
print('$v', d['ms_per_step'], {n:k[n] for n in ('part_scatter','group_sums','cross','gram_resid','gram_design','seg_build','cluster_sort','cluster_fix','layout_scatter') if n in k})"
  done
done
