"""BASELINE.json configs 2, 3 and 4 as parity cases against the C restatement of
the reference loop (oracle/altproj_c.c): config 2 at its full size (10M rows), the
headline config 3 at its full size (50M rows, k = 10, HC1: the bench's workload),
config 4 (three high-cardinality FEs, two-way clustered SE) at 5M rows.  Integer
outputs must be equal, beta and IID/HC1 SE within 1e-10 relative; the two-way
CGM cluster counts must equal the host's distinct counts."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.parametrize("cfg,n", [(2, 10_000_000), (3, 50_000_000), (4, 5_000_000)])
def test_baseline_config_vs_c_oracle(cfg, n):
    import config_runs

    if cfg == 2:
        line = config_runs.run(2, n, 5, [100_000, 1_000], "iid")
    elif cfg == 3:
        line = config_runs.run(3, n, 10, [100_000, 1_000], "HC1")
    else:
        line = config_runs.run(4, n, 10, [1_000_000, 100_000, 10_000], "cluster", cluster_fes=[1, 2])
        from leanfe_amd import synth

        d = synth.panel(n, 0, [1_000_000, 100_000, 10_000], seed=12345)
        keep = np.ones(n, dtype=bool)
        for f in (1, 2, 3):  # single-pass singleton drop on pre-filter counts
            c = d[f"fe{f}"]
            keep &= np.bincount(c, minlength=c.max() + 1)[c] > 1
        g2 = np.unique(d["fe2"][keep]).size
        g3 = np.unique(d["fe3"][keep]).size
        g23 = np.unique(d["fe2"][keep].astype(np.int64) * 10_000 + d["fe3"][keep]).size
        assert line["cluster_G"] == [g2, g3, g23]
        assert line["cluster_se_finite_positive"]
    assert line["ints_equal"]
    assert line["max_rel_beta"] < 1e-10
    assert line["max_rel_se"] < 1e-10
