"""HBM traffic per launch of each engine kernel from rocprofv3 PMC passes.

Reads gpurun_out/pmc/{fetch,write}/run_counter_collection.csv (tools/pmc.sh, one
counter per pass, never combined with tracing) and writes a JSON keyed by the
engine's kernel ids (the names bench.py reports):

    bytes = 2 * FETCH_SIZE + WRITE_SIZE        (KiB in the CSV)

FETCH_SIZE is doubled per MI355X_MICROARCH.md "HBM": on gfx950 it reports half
the bytes of a wide streaming read.  Launches of the timed steps are averaged.

    python tools/pmc_traffic.py gpurun_out/pmc profiles/r01/pmc_traffic.json --rows 50000000 --k 10 \
        --levels 100000,1000 --vcov HC1
"""
import argparse
import csv
import json
import os
import re
from collections import defaultdict

# engine kernel id -> demangled kernel name prefix
KERNELS = {
    "part_hist": ("k_part_hist",), "part_scatter": ("k_part_scatter",), "mark": ("k_mark",),
    "group_sums": ("k_sums4", "k_sums2_raw"), "tp": ("k_tp",), "tq": ("k_tq",),
    "gram_design": ("k_design_rows", "k_gram<0,"), "gram_resid": ("k_resid_rows", "k_gram<1,"),
    "gram_tables": ("k_tables_gram",), "layout_sort": ("k_ls_scatter",),
}

ap = argparse.ArgumentParser()
ap.add_argument("pmc_dir")
ap.add_argument("out")
ap.add_argument("--rows", type=int, required=True)
ap.add_argument("--k", type=int, required=True)
ap.add_argument("--levels", required=True)
ap.add_argument("--vcov", required=True)
a = ap.parse_args()


def per_kernel(counter):
    vals = defaultdict(list)
    f = os.path.join(a.pmc_dir, counter.lower().split("_")[0], "run_counter_collection.csv")
    per = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        per[d] += float(r["Counter_Value"])
        names[d] = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("lfe::", "").replace(" ", "")
    for d, v in per.items():
        vals[names[d]].append(v * 1024.0)
    return vals


fetch, write = per_kernel("FETCH_SIZE"), per_kernel("WRITE_SIZE")
out = {"config": {"rows": a.rows, "k": a.k, "levels": [int(x) for x in a.levels.split(",")], "vcov": a.vcov},
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes); bytes = 2*FETCH + WRITE",
       "kernels": {}}
for kid, prefix in KERNELS.items():
    fk = [n for n in fetch if any(n.startswith(px.replace(" ", "")) for px in prefix)]
    if not fk:
        continue
    fv = [v for n in fk for v in fetch[n]]
    wv = [v for n in fk for v in write.get(n, [])]
    # the timed steps are the last launches; use the median launch
    fv.sort()
    wv.sort()
    fb = fv[len(fv) // 2]
    wb = wv[len(wv) // 2] if wv else 0.0
    out["kernels"][kid] = {"fetch_bytes": 2 * fb, "write_bytes": wb, "bytes_per_launch": 2 * fb + wb,
                           "launches_profiled": len(fv), "kernel": fk[0]}
json.dump(out, open(a.out, "w"), indent=1)
print(json.dumps(out["kernels"], indent=1))
