"""Per-kernel table from tools/pmc.sh output (gpurun_out/pmc/<pass>/run_counter_collection.csv).

Averages each counter over the dispatches of a kernel (the last `--last` dispatches,
i.e. the timed steps).  FETCH_SIZE is doubled (gfx950 reports half the bytes of a
wide streaming read, MI355X_MICROARCH.md "HBM"); sizes in the CSV are in KiB.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [per dispatch]
dur = defaultdict(list)
for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
    per = defaultdict(lambda: defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("lfe::", "")
        d = int(r["Dispatch_Id"])
        per[(k, d)][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[(k, d)] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    for (k, d), cs in per.items():
        for c, v in cs.items():
            vals[k][c].append(v)
        if "FETCH_SIZE" in cs:
            dur[k].append(meta[(k, d)])

want = ["ms", "FETCH_GB", "WRITE_GB", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
        "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "L2hit"]
if len(sys.argv) > 2:
    want = ["ms"] + sys.argv[2].split(",")
print("%-28s" % "kernel" + "".join("%14s" % w[-14:] for w in want))
n_show = 14
for k in sorted(vals, key=lambda k: -sum(dur.get(k, [0])) / max(len(dur.get(k, [1])), 1))[:n_show]:
    cs = vals[k]
    avg = lambda c: sum(cs[c]) / len(cs[c]) if cs.get(c) else float("nan")
    row = {
        "ms": sum(dur[k]) / len(dur[k]) if dur.get(k) else float("nan"),
        "FETCH_GB": 2 * avg("FETCH_SIZE") * 1024 / 1e9,
        "WRITE_GB": avg("WRITE_SIZE") * 1024 / 1e9,
    }
    for c in want:
        if c not in row and c != "L2hit":
            row[c] = avg(c)
    h, m = avg("TCC_HIT_sum"), avg("TCC_MISS_sum")
    if "L2hit" in want:
        row["L2hit"] = h / (h + m) if h + m else float("nan")
    print("%-28s" % k[:28] + "".join("%14.4g" % row[w] for w in want))
