"""CPU: the oracle (oracle/altproj.py) against the golden fixtures.

Golden ``ref_*`` values were computed by the reference's own NumPy/SciPy code
(exact LSDV solve + compute_se_compress, see tests/golden/make_golden.py);
``oracle_*`` values are the oracle at the reference defaults and pin the
iteration count / integer outputs for the GPU parity tests."""
import numpy as np
import pytest

from golden_util import load, names, ncl
from oracle import altproj, yoco

YOCO_CASES = [n for n in names() if load(n)[0]["pinned"] == "reference-yoco"]
CASES = [n for n in names() if n not in YOCO_CASES]


def _fit(meta, data, **kw):
    return altproj.fit(data, meta["y"], meta["xs"], meta["fes"], strategy=meta["strategy"],
                       weights=meta["weights"], vcov=meta["vcov"], cluster_cols=meta["cluster_cols"],
                       ssc=meta["ssc"], instruments=meta.get("instruments"), **kw)


def test_fixture_count():
    assert len(CASES) >= 15 and len(YOCO_CASES) >= 7


@pytest.mark.parametrize("name", YOCO_CASES)
def test_yoco_oracle_matches_reference_functions(name):
    """strategy='compress': the oracle's group-by + LSDV WLS + grouped-RSS SEs == the
    reference's own build_design_matrix / solve_wls / compute_rss_grouped /
    compute_se_compress on the same records (tests/golden/make_golden.py)."""
    meta, data, exp = load(name)
    r = yoco.fit(data, meta["y"], meta["xs"], meta["fes"], weights=meta["weights"], vcov=meta["vcov"],
                 cluster_cols=meta["cluster_cols"], ssc=meta["ssc"])
    assert r["n_obs"] == int(exp["oracle_n_obs"]) and r["df_resid"] == int(exp["oracle_df_resid"])
    assert r["n_compressed"] == int(exp["oracle_n_compressed"])
    np.testing.assert_allclose(r["beta"], exp["ref_beta"], rtol=1e-11, atol=0)
    np.testing.assert_allclose(r["se"], exp["ref_se"], rtol=1e-11, atol=0)
    np.testing.assert_allclose(r["rss"], exp["ref_rss"], rtol=1e-11)
    assert ncl(r["n_clusters"]) == ncl(meta["ref_n_clusters"])


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_stored_outputs(name):
    meta, data, exp = load(name)
    r = _fit(meta, data, demean_tol=meta["demean_tol"], max_iter=meta["max_iter"])
    assert r["iterations"] == int(exp["oracle_iterations"])
    assert r["n_obs"] == int(exp["oracle_n_obs"])
    assert r["df_resid"] == int(exp["oracle_df_resid"])
    assert tuple(r["fe_dims"]) == tuple(exp["oracle_fe_dims"].tolist())
    np.testing.assert_allclose(r["beta"], exp["oracle_beta"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(r["se"], exp["oracle_se"], rtol=1e-12, atol=0)
    assert ncl(r["n_clusters"]) == ncl(meta["oracle_n_clusters"])


@pytest.mark.parametrize("name", [n for n in CASES if load(n)[0]["pinned"] == "reference-lsdv"])
def test_oracle_converged_matches_reference_lsdv(name):
    """Oracle iterated to machine precision == the reference's exact LSDV fit."""
    meta, data, exp = load(name)
    r = _fit(meta, data, demean_tol=1e-14, max_iter=100000)
    np.testing.assert_allclose(r["beta"], exp["ref_beta"], rtol=1e-9, atol=0)
    np.testing.assert_allclose(r["se"], exp["ref_se"], rtol=1e-9, atol=0)
    assert ncl(r["n_clusters"]) == ncl(meta["ref_n_clusters"])


@pytest.mark.parametrize("name", [n for n in CASES if load(n)[0]["pinned"] == "reference-wls-beta"])
def test_weighted_oracle_converged_matches_reference_wls(name):
    """Weighted fits: the oracle iterated to machine precision gives the reference's exact
    weighted LSDV beta (its solve_wls with per-row sqrt-weights, compress.py:659-680).  The
    stop test is unweighted (polars_impl.py:513), so a weighted fit never meets a 1e-14 tol:
    3000 sweeps reach the rounding floor on these panels."""
    meta, data, exp = load(name)
    r = _fit(meta, data, demean_tol=1e-14, max_iter=3000)
    np.testing.assert_allclose(r["beta"], exp["ref_beta"], rtol=1e-9, atol=0)


@pytest.mark.parametrize("name", [n for n in CASES if load(n)[0]["pinned"] == "reference-lsdv"])
def test_default_tolerance_close_to_reference(name):
    """At the reference defaults (tol 1e-6, max_iter 50) alt-proj stops within
    1e-7 relative of the exact LSDV solution on these panels (convergence error)."""
    meta, data, exp = load(name)
    np.testing.assert_allclose(exp["oracle_beta"], exp["ref_beta"], rtol=1e-7, atol=0)
    np.testing.assert_allclose(exp["oracle_se"], exp["ref_se"], rtol=1e-7, atol=0)


@pytest.mark.parametrize("name", [n for n in CASES if load(n)[0]["pinned"] == "reference-iv"])
def test_oracle_iv_matches_reference_functions(name):
    """IV/2SLS: the oracle's 2SLS and IV SEs == the reference's own common.iv_2sls and
    std_errors._compute_se_*_iv evaluated on the same demeaned columns."""
    meta, data, exp = load(name)
    assert meta["instruments"]
    r = _fit(meta, data, demean_tol=meta["demean_tol"], max_iter=meta["max_iter"])
    np.testing.assert_allclose(r["beta"], exp["ref_beta"], rtol=1e-11, atol=0)
    np.testing.assert_allclose(r["se"], exp["ref_se"], rtol=1e-11, atol=0)
    assert ncl(r["n_clusters"]) == ncl(meta["ref_n_clusters"])


def test_singleton_rule_is_single_pass():
    # fe1 = [0,0,1,2,2], fe2 = [0,1,1,2,2]: pass 1 drops rows with fe1 level 1 (row 2)
    # and rows whose fe2 level is a singleton (row 0: fe2=0 count 1).  After the
    # drop fe2 level 1 becomes a singleton (row 1) but is NOT dropped again.
    keep = altproj.singleton_keep([np.array([0, 0, 1, 2, 2]), np.array([0, 1, 1, 2, 2])], [3, 3])
    assert keep.tolist() == [False, True, False, True, True]


def test_weighted_check_is_unweighted():
    """polars_impl.py:512-521 checks UNweighted y means even with weights, so a
    weighted fit on an unbalanced panel runs to max_iter (fixture panel_w_cl1)."""
    meta, data, exp = load("panel_w_cl1")
    assert int(exp["oracle_iterations"]) == meta["max_iter"]
