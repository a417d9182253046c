"""End-to-end leanfe(backend="hip") from host NumPy columns: formula, factorization
(sparse int64 ids go to the device), H2D load, strategy 'auto' (exact distinct-row
count on the device), solve, SEs.  Prints one JSON line with the wall time and the
engine's phase timings.

    python tools/e2e.py [--rows 50000000] [--vcov HC1] [--sparse-ids]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from leanfe_amd import hip_impl, leanfe_hip, synth  # noqa: E402

hip_impl.KNOBS["phase_timing"] = True  # the per-phase device times in the printed lines


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=50_000_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--levels", default="100000,1000")
    ap.add_argument("--vcov", default="HC1")
    ap.add_argument("--sparse-ids", action="store_true", help="FE ids as sparse int64 (device factorization)")
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--parquet", default=None, help="also time leanfe(<this Parquet path>): streamed and read whole")
    a = ap.parse_args()
    levels = [int(x) for x in a.levels.split(",")]
    t0 = time.perf_counter()
    data = synth.panel(a.rows, a.k, levels, seed=12345)
    if a.sparse_ids:
        for f in range(len(levels)):
            data[f"fe{f + 1}"] = data[f"fe{f + 1}"].astype(np.int64) * 7_919_000_011 + 123
    t_gen = time.perf_counter() - t0
    xs = " + ".join(f"x{j + 1}" for j in range(a.k))
    fes = " + ".join(f"fe{f + 1}" for f in range(len(levels)))
    formula = f"y ~ {xs} | {fes}"
    out = []
    for _ in range(a.repeat):
        t0 = time.perf_counter()
        r = leanfe_hip(data, formula=formula, vcov=a.vcov, quiet=True)
        out.append(time.perf_counter() - t0)
    print(json.dumps(dict(rows=a.rows, k=a.k, levels=levels, vcov=a.vcov, sparse_ids=a.sparse_ids,
                          wall_s=[round(t, 3) for t in out], gen_s=round(t_gen, 2), iterations=r.iterations,
                          compression_ratio=r.compression_ratio,
                          timings={k: round(v, 4) for k, v in r.timings.items()})), flush=True)
    if a.parquet:
        import pyarrow as pa
        import pyarrow.parquet as pq
        t0 = time.perf_counter()
        pq.write_table(pa.table(data), a.parquet, row_group_size=1 << 20)
        t_write = time.perf_counter() - t0
        del data
        for mode in ("1", "0"):  # streamed (lfe_load_rows per batch) / read whole, then lfe_load
            hip_impl.KNOBS["stream"] = mode == "1"
            walls = []
            for _ in range(a.repeat):
                t0 = time.perf_counter()
                r = leanfe_hip(a.parquet, formula=formula, vcov=a.vcov, strategy="alt_proj", quiet=True)
                walls.append(time.perf_counter() - t0)
            print(json.dumps(dict(rows=a.rows, parquet=True, streamed=mode == "1", write_s=round(t_write, 2),
                                  wall_s=[round(t, 3) for t in walls], mrows_s=round(a.rows / min(walls) / 1e6, 1),
                                  load_s=round(r.timings["load_s"], 3), iterations=r.iterations)), flush=True)


if __name__ == "__main__":
    main()
