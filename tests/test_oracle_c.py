"""The C restatement (oracle/altproj_c.c, bench.py's CPU baseline) against the
golden fixtures' oracle outputs: same iterations / n_obs / df_resid, beta and SE
to 1e-10 (unweighted IID and HC1 fixtures)."""
from __future__ import annotations

import shutil

import numpy as np
import pytest

from golden_util import load, names

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")

CASES = [n for n in names() if n.endswith(("_iid", "_hc1")) and "_w_" not in n and load(n)[0]["strategy"] not in ("demean", "compress")
         and not load(n)[0].get("instruments")]  # the C port is the OLS baseline only


@pytest.mark.parametrize("name", CASES)
def test_c_oracle_matches_golden(name):
    from oracle.altproj_c import fit_c

    meta, data, exp = load(name)
    cols = [data[meta["y"]]] + [data[x] for x in meta["xs"]]
    codes, levels = [], []
    for f in meta["fes"]:
        u, inv = np.unique(data[f], return_inverse=True)
        codes.append(inv.astype(np.int32))
        levels.append(len(u))
    r = fit_c(cols, codes, levels, vcov=meta["vcov"], tol=meta["demean_tol"], max_iter=meta["max_iter"], threads=4)
    assert r["iterations"] == int(exp["oracle_iterations"])
    assert r["n_obs"] == int(exp["oracle_n_obs"])
    assert r["df_resid"] == int(exp["oracle_df_resid"])
    np.testing.assert_allclose(r["beta"], exp["oracle_beta"], rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(r["se"], exp["oracle_se"], rtol=1e-10, atol=1e-14)
