"""cProfile of one warm leanfe(backend="hip") call on the 50M-row headline panel from host NumPy
(where the end-to-end time beyond the H2D copy and the solve goes).

    python tools/e2e_profile.py [--rows 50000000] [--sparse-ids]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from leanfe_amd import leanfe_hip, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=50_000_000)
    ap.add_argument("--sparse-ids", action="store_true")
    a = ap.parse_args()
    levels = [100_000, 1_000]
    data = synth.panel(a.rows, 10, levels, seed=12345)
    if a.sparse_ids:
        for f in range(len(levels)):
            data[f"fe{f + 1}"] = data[f"fe{f + 1}"].astype(np.int64) * 7_919_000_011 + 123
    formula = "y ~ " + " + ".join(f"x{j + 1}" for j in range(10)) + " | fe1 + fe2"
    leanfe_hip(data, formula=formula, vcov="HC1", quiet=True)  # warm
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    r = leanfe_hip(data, formula=formula, vcov="HC1", quiet=True)
    pr.disable()
    wall = time.perf_counter() - t0
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(35)
    print(f"wall {wall:.4f} s; timings {r.timings}")
    print(s.getvalue())


if __name__ == "__main__":
    main()
