"""Out-of-core X (data larger than HBM): the FE codes stay resident, the
columns are streamed in row chunks (lfe_load_codes + lfe_stream_*, hip_impl._out_of_core_fit).
The streamed fit must equal the CPU restatement of the reference (oracle/altproj.py,
polars_impl.py:468-537 + std_errors.py:183-282) at the usual bars - integers equal, beta and
SE within 1e-10 - for every chunking, with singletons dropped, when the Gram from the tables
trips its guard (pass 3), from a Parquet file, and bit-identically run to run."""
from __future__ import annotations

import numpy as np
import pytest

from leanfe_amd import synth
from oracle import altproj

pytestmark = pytest.mark.gpu


def _panel(n, k, L, seed, singletons=0):
    d = synth.panel(n, k, L, seed=seed)
    if singletons:  # rows alone in a primary level: the single-pass drop removes them
        rng = np.random.default_rng(seed)
        idx = rng.choice(n, singletons, replace=False)
        fe1 = np.array(d["fe1"], copy=True)
        fe1[idx] = L[0] + np.arange(singletons)
        d["fe1"] = fe1
    return d


def _check(r, o, xs):
    assert r.iterations == o["iterations"] and r.n_obs == o["n_obs"] and r.df_resid == o["df_resid"]
    assert list(r.fe_dims) == list(o["fe_dims"])
    b = np.array([r.coefs[x] for x in xs])
    s = np.array([r.std_errors[x] for x in xs])
    np.testing.assert_allclose(b, o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(s, o["se"], rtol=1e-10, atol=0)
    return b, s


@pytest.mark.parametrize("vcov,chunk", [("HC1", 131_071), ("iid", 1 << 20), ("HC1", 999_999_999)])
def test_streamed_fit_matches_oracle(vcov, chunk):
    from leanfe_amd import leanfe_hip
    n, k, L = 1_000_003, 5, [20_000, 400]
    d = _panel(n, k, L, seed=5, singletons=37)
    xs = [f"x{j + 1}" for j in range(k)]
    o = altproj.fit(d, "y", xs, ["fe1", "fe2"], vcov=vcov)
    r = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], strategy="alt_proj", vcov=vcov, quiet=True,
                   out_of_core=True, chunk_rows=chunk)
    _check(r, o, xs)


def test_streamed_design_pass_when_the_tables_guard_trips():
    """A column the FEs explain almost entirely: the tables Gram's guard trips, lfe_gram returns
    LFE_ENEEDPASS and the streamed design-Gram pass (pass 3) runs."""
    from leanfe_amd import leanfe_hip
    n, L = 400_000, [20_000, 300]
    d = synth.panel(n, 3, L, seed=61)
    eff = np.random.default_rng(61).normal(0, 1, L[0])
    d["x1"] = d["x1"] + 1e3 * eff[d["fe1"]]
    xs = ["x1", "x2", "x3"]
    o = altproj.fit(d, "y", xs, ["fe1", "fe2"], vcov="HC1")
    from leanfe_amd._lib import Engine
    with Engine(0) as eng:
        eng.profile(True)
        r = leanfe_hip(d, y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], strategy="alt_proj", vcov="HC1",
                       quiet=True, engine=eng, out_of_core=True, chunk_rows=65_536)
        ks = eng.kernel_stats()
    assert "gram_design" in ks, sorted(ks)
    _check(r, o, xs)


def test_streamed_parquet_and_bit_identical_reruns(tmp_path):
    import pyarrow as pa
    import pyarrow.parquet as pq

    from leanfe_amd import leanfe_hip
    n, k, L = 600_000, 4, [9_000, 250]
    d = synth.panel(n, k, L, seed=9)
    path = str(tmp_path / "panel.parquet")
    pq.write_table(pa.table({c: np.asarray(v) for c, v in d.items()}), path, row_group_size=100_000)
    xs = [f"x{j + 1}" for j in range(k)]
    o = altproj.fit(d, "y", xs, ["fe1", "fe2"], vcov="HC1")
    runs = [leanfe_hip(path, y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], strategy="alt_proj", vcov="HC1",
                       quiet=True, out_of_core=True, chunk_rows=70_000) for _ in range(2)]
    b0, s0 = _check(runs[0], o, xs)
    b1, s1 = _check(runs[1], o, xs)
    np.testing.assert_array_equal(b0, b1)
    np.testing.assert_array_equal(s0, s1)


def test_streamed_synthetic_chunks_match_the_resident_solve():
    """The engine API on the device-generated panel (benchmark path): codes resident, columns
    generated chunk by chunk - the same fit as the resident solve (bench.solve_step)."""
    import bench
    from leanfe_amd import inference
    from leanfe_amd._lib import Engine
    n, k, L = 3_000_000, 10, [100_000, 1_000]
    beta = synth.betas(k)
    with Engine(0) as eng:
        eng.synth_load(n, k, L, beta, seed=77)
        ref = bench.solve_step(eng, "hc1")
    with Engine(0) as eng:
        eng.synth_load_codes(n, k, L, seed=77)
        n_obs, dims, card = eng.drop_singletons()
        eng.stream_synth_pass(1, k, L, beta, chunk_rows=400_000, seed=77)
        it, _ = eng.demean(sorted(range(2), key=lambda i: card[i]), 1e-6, 50, check_from=3)
        G = eng.gram()
        XtX, Xty = inference.split_gram(G)
        bf, XtX_inv = inference.solve_normal(XtX, Xty)
        out = eng.stream_synth_pass(2, k, L, beta, chunk_rows=400_000, seed=77, beta_full=bf)
        df = n_obs - (k + 1) - (sum(dims) - 2)
        se = inference.se_hc1(XtX_inv[1:, 1:], out[4:4 + k * k].reshape(k, k), n_obs, df)
    assert it == ref["iterations"] and n_obs == ref["n_obs"] and df == ref["df_resid"]
    np.testing.assert_allclose(bf[1:], ref["beta"], rtol=1e-11, atol=0)
    np.testing.assert_allclose(se, ref["se"], rtol=1e-11, atol=0)
    assert out[1] == pytest.approx(ref["rss"], rel=1e-11)
