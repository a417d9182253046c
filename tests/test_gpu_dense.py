"""Dense count-table cross terms (leanfe_amd/csrc/lfe_dense.hip).

For two FEs the sweep's cross terms T_P = N alpha_Q and T_Q = N' alpha_P (N[h][q] = kept rows with
codes (h, q) per bucket of the primary FE) run on the matrix cores when the table holds >= 0.3
rows per cell; otherwise the segment / run layouts of lfe_iter.hip gather row by row.  Both are
restatements of the same projection loop (polars_impl.py:490-526), so:
- each path matches the CPU oracle (oracle/altproj.py) at 1e-10 with equal `iterations`;
- the two paths agree with each other to rounding;
- the dense path repeats bit for bit;
- a panel whose (h, q) pairs hold more than 255 rows takes the build's 16-bit recount (its 8-bit
  counters overflow) and still matches the oracle;
- an owner shard (strong scaling, few buckets) takes it too;
- the exact integer form (i8 count tables x base-128 digits of the effects on
  v_mfma_i32_16x16x64_i8, the default) agrees with the f64-MFMA form (LFE_DN8=0) to rounding,
  including blocks with cells over 127 rows (summed in f64 from their u16 counts).
LFE_DENSE=1 forces the dense path wherever it fits, LFE_DENSE=0 turns it off."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _fit(data, xs, vcov="HC1"):
    from leanfe_amd import leanfe_hip

    r = leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], strategy="alt_proj", vcov=vcov, quiet=True,
                   device=0)
    return (np.array([r.coefs[x] for x in xs]), np.array([r.std_errors[x] for x in xs]), r.iterations, r.n_obs,
            r.df_resid)


def _oracle(data, xs, vcov="HC1"):
    from oracle import altproj

    return altproj.fit(data, "y", xs, ["fe1", "fe2"], vcov=vcov)


def _check(res, o):
    b, s, it, n_obs, df = res
    assert it == o["iterations"] and n_obs == o["n_obs"] and df == o["df_resid"], (it, o["iterations"])
    np.testing.assert_allclose(b, o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(s, o["se"], rtol=1e-10, atol=0)


@pytest.mark.parametrize("vcov", ["HC1", "iid"])
def test_dense_and_row_paths_match_oracle_and_each_other(vcov, knob):
    from leanfe_amd import synth

    k = 5
    xs = [f"x{j + 1}" for j in range(k)]
    # 0.6 rows per cell: the default picks the dense path
    data = synth.panel(1_200_000, k, [4_000, 500], seed=2024)
    o = _oracle(data, xs, vcov)
    knob.setenv("LFE_DENSE", "0")
    rows = _fit(data, xs, vcov)
    knob.delenv("LFE_DENSE")
    dense = _fit(data, xs, vcov)
    _check(rows, o)
    _check(dense, o)
    np.testing.assert_allclose(dense[0], rows[0], rtol=1e-13, atol=0)
    again = _fit(data, xs, vcov)
    np.testing.assert_array_equal(dense[0], again[0])
    np.testing.assert_array_equal(dense[1], again[1])


def test_dense_with_singletons_and_ragged_bucket(knob):
    """Singleton rows dropped before the table is built (40 primary levels with one row each); a
    primary FE whose last bucket is partial (G_P = 3,041) and a secondary FE that is not a multiple
    of 16 levels (G_Q = 77)."""
    from leanfe_amd import synth

    k = 3
    xs = [f"x{j + 1}" for j in range(k)]
    data = synth.panel(300_000, k, [3_001, 77], seed=5)
    fe1 = np.array(data["fe1"], copy=True)
    fe1[:40] = np.arange(40) + 3_001  # 40 new levels of one row each: singletons, dropped
    data = dict(data, fe1=fe1)
    knob.setenv("LFE_DENSE", "1")
    _check(_fit(data, xs), _oracle(data, xs))


def test_dense_counts_beyond_8_bits(knob):
    """(h, q) pairs with ~50K rows: on the 8-bit counters of the build (forced with LFE_DN_C8=1: at
    1,000 primary levels the build would otherwise pick 16-bit chunks, since 8-bit ones would leave
    CUs idle) these pairs overflow, and the chunk is counted again on 16-bit counters.  A wrapped
    count would move beta far from the oracle; the recounted table gives the same bits as the build
    that starts on 16-bit counters, and agrees with the row layouts (LFE_DENSE=0) at 1e-13."""
    rng = np.random.default_rng(11)
    n, k = 400_000, 3
    fe1 = rng.integers(0, 1_000, n).astype(np.int32)
    fe2 = rng.integers(0, 40, n).astype(np.int32)
    heavy = rng.random(n) < 0.25  # a quarter of the rows on two (h, q) pairs: ~50K rows each
    fe1[heavy] = np.where(rng.random(heavy.sum()) < 0.5, 7, 700).astype(np.int32)
    fe2[heavy] = 3
    x = rng.standard_normal((n, k))
    a1 = rng.standard_normal(1_000)
    a2 = rng.standard_normal(40)
    y = x @ np.array([1.0, -0.5, 0.25]) + a1[fe1] + a2[fe2] + rng.standard_normal(n)
    data = {"y": y, "fe1": fe1, "fe2": fe2, **{f"x{j + 1}": x[:, j].copy() for j in range(k)}}
    xs = ["x1", "x2", "x3"]
    o = _oracle(data, xs)
    knob.setenv("LFE_DENSE", "1")
    knob.setenv("LFE_DN_C8", "1")
    dense8 = _fit(data, xs)
    _check(dense8, o)
    knob.setenv("LFE_DN_C8", "0")
    dense16 = _fit(data, xs)
    np.testing.assert_array_equal(dense8[0], dense16[0])
    np.testing.assert_array_equal(dense8[1], dense16[1])
    knob.delenv("LFE_DN_C8")
    knob.setenv("LFE_DENSE", "0")
    rows = _fit(data, xs)
    _check(rows, o)
    np.testing.assert_allclose(dense8[0], rows[0], rtol=1e-13, atol=0)


def test_dense_owner_shard_matches_whole_panel(knob):
    """Rank 7 of 8 of the strong-scaled headline schedule solved alone (bench --emulate-rank): its
    few buckets take the dense path and the owner shard matches the oracle on the same rows."""
    import bench
    from leanfe_amd import synth
    from leanfe_amd._lib import Engine
    from oracle import altproj

    n, k, L = 2_000_000, 4, [40_000, 300]
    knob.setenv("LFE_DENSE", "1")
    with Engine(0) as eng:
        eng.synth_load_owned(n, k, L, synth.betas(k), 0, 35_000, 40_000, seed=31)
        got = bench.solve_step(eng, "iid")
        again = bench.solve_step(eng, "iid")
    np.testing.assert_array_equal(got["beta"], again["beta"])
    data = synth.panel(n, k, L, seed=31)
    keep = (data["fe1"] >= 35_000) & (data["fe1"] < 40_000)
    sub = {c: np.asarray(v)[keep] for c, v in data.items()}
    o = altproj.fit(sub, "y", [f"x{j + 1}" for j in range(k)], ["fe1", "fe2"], vcov="iid")
    assert got["iterations"] == o["iterations"]
    np.testing.assert_allclose(got["beta"], o["beta"], rtol=1e-10, atol=0)
    np.testing.assert_allclose(got["se"], o["se"], rtol=1e-10, atol=0)


@pytest.mark.parametrize("vcov,p_k", [("HC1", 10), ("iid", 3), ("HC1", 15)])
def test_dense_i8_digits_match_f64_mfma_and_oracle(vcov, p_k, knob):
    """The i8 passes (default) against the f64-MFMA passes (LFE_DN8=0) and the oracle: equal
    integers, beta / SE at 1e-10 of the oracle and 1e-12 of each other, bit-identical repeats;
    k = 15 fills all 16 MFMA columns (p = 16)."""
    from leanfe_amd import synth

    xs = [f"x{j + 1}" for j in range(p_k)]
    data = synth.panel(900_000, p_k, [3_000, 600], seed=77)
    o = _oracle(data, xs, vcov)
    knob.setenv("LFE_DENSE", "1")
    knob.setenv("LFE_DN8", "0")
    f64 = _fit(data, xs, vcov)
    knob.delenv("LFE_DN8")
    i8 = _fit(data, xs, vcov)
    _check(f64, o)
    _check(i8, o)
    np.testing.assert_allclose(i8[0], f64[0], rtol=1e-12, atol=0)
    np.testing.assert_allclose(i8[1], f64[1], rtol=1e-12, atol=0)
    again = _fit(data, xs, vcov)
    np.testing.assert_array_equal(i8[0], again[0])
    np.testing.assert_array_equal(i8[1], again[1])


def test_dense_i8_flagged_blocks_mixed_with_exact_blocks(knob):
    """A few (h, q) pairs with 128-400 rows among ordinary cells: their 16 x 64 blocks are flagged
    (zero in the i8 tables, u16 counts summed in f64) while every other block runs on the i8
    MFMAs - both orientations (K1 and K2 blocks) - against the oracle and the f64 passes."""
    rng = np.random.default_rng(5)
    n, k = 600_000, 4
    fe1 = rng.integers(0, 2_000, n).astype(np.int32)
    fe2 = rng.integers(0, 300, n).astype(np.int32)
    pairs = [(17, 5, 128), (900, 299, 400), (1_500, 64, 200), (1_999, 0, 131)]
    i0 = 0
    for h, q, m in pairs:
        fe1[i0:i0 + m] = h
        fe2[i0:i0 + m] = q
        i0 += m
    x = rng.standard_normal((n, k))
    y = x @ np.linspace(1.0, 0.2, k) + rng.standard_normal(2_000)[fe1] + rng.standard_normal(300)[fe2] + \
        rng.standard_normal(n)
    data = {"y": y, "fe1": fe1, "fe2": fe2, **{f"x{j + 1}": x[:, j].copy() for j in range(k)}}
    xs = [f"x{j + 1}" for j in range(k)]
    o = _oracle(data, xs)
    knob.setenv("LFE_DENSE", "1")
    i8 = _fit(data, xs)
    _check(i8, o)
    knob.setenv("LFE_DN8", "0")
    f64 = _fit(data, xs)
    np.testing.assert_allclose(i8[0], f64[0], rtol=1e-12, atol=0)


def test_dense_four_bit_counters(knob):
    """The 256-group chunks on 4-bit counters (LFE_DN_C4=1): a sparse panel's tables are the same
    bits as the 8-bit build's, and a panel with cells of 16+ rows (two ~50K-row pairs and many
    2-16-row ones) recounts those chunks on 8- and 16-bit counters and still matches the oracle."""
    from leanfe_amd import synth

    xs = ["x1", "x2", "x3"]
    data = synth.panel(1_000_000, 3, [4_096, 1_000], seed=13)
    knob.setenv("LFE_DENSE", "1")
    knob.setenv("LFE_DN_C4", "1")
    c4 = _fit(data, xs)
    knob.setenv("LFE_DN_C4", "0")
    c8 = _fit(data, xs)
    np.testing.assert_array_equal(c4[0], c8[0])
    np.testing.assert_array_equal(c4[1], c8[1])
    _check(c4, _oracle(data, xs))
    rng = np.random.default_rng(17)
    n = 400_000
    fe1 = rng.integers(0, 1_024, n).astype(np.int32)
    fe2 = rng.integers(0, 40, n).astype(np.int32)
    heavy = rng.random(n) < 0.25
    fe1[heavy] = np.where(rng.random(heavy.sum()) < 0.5, 7, 700).astype(np.int32)
    fe2[heavy] = 3
    x = rng.standard_normal((n, 3))
    y = x @ np.array([1.0, -0.5, 0.25]) + rng.standard_normal(1_024)[fe1] + rng.standard_normal(40)[fe2] + \
        rng.standard_normal(n)
    heavy_data = {"y": y, "fe1": fe1, "fe2": fe2, **{f"x{j + 1}": x[:, j].copy() for j in range(3)}}
    knob.setenv("LFE_DN_C4", "1")
    _check(_fit(heavy_data, xs), _oracle(heavy_data, xs))


@pytest.mark.parametrize("vcov,p_k", [("HC1", 14), ("iid", 20), ("HC1", 20)])
def test_dense_wide_fits(vcov, p_k, knob):
    """Two FEs at p = 15 and 21: the dense passes in 16-column groups (the row layouts' LDS tables
    do not fit), the column-group group sums and the Gram from the group tables (raw MFMA pass +
    table terms) against the oracle and the general sweeps (LFE_DENSE=0), bit-identical repeats."""
    from leanfe_amd import synth

    xs = [f"x{j + 1}" for j in range(p_k)]
    data = synth.panel(900_000, p_k, [3_000, 600], seed=91)
    o = _oracle(data, xs, vcov)
    dense = _fit(data, xs, vcov)
    _check(dense, o)
    again = _fit(data, xs, vcov)
    np.testing.assert_array_equal(dense[0], again[0])
    np.testing.assert_array_equal(dense[1], again[1])
    knob.setenv("LFE_DENSE", "0")
    rows = _fit(data, xs, vcov)
    _check(rows, o)
    np.testing.assert_allclose(dense[0], rows[0], rtol=1e-11, atol=0)
    np.testing.assert_allclose(dense[1], rows[1], rtol=1e-11, atol=0)


def test_two_fe_column_group_sums_form_their_own_raw_gram(knob):
    """a two-FE fit whose secondary table does not fit LDS (p = 14, G_Q = 2,000)
    takes the column-group sums, which form no raw Gram tile; the Gram must not reuse a tile left
    by an earlier fit on the same Engine (here a G_Q = 600 fit, whose sums do write one).  Both
    fits against the oracle, the second also against the sums without column groups
    (LFE_SUMS_CG=0) and repeated on the same Engine."""
    from leanfe_amd import leanfe_hip, synth
    from leanfe_amd._lib import Engine

    k = 13
    xs = [f"x{j + 1}" for j in range(k)]
    first = synth.panel(600_000, k, [3_000, 600], seed=92)
    wide = synth.panel(1_000_000, k, [6_000, 2_000], seed=93)

    def fit(data, eng):
        r = leanfe_hip(data, y_col="y", x_cols=xs, fe_cols=["fe1", "fe2"], strategy="alt_proj", vcov="HC1",
                       quiet=True, engine=eng)
        return (np.array([r.coefs[x] for x in xs]), np.array([r.std_errors[x] for x in xs]), r.iterations, r.n_obs,
                r.df_resid)

    o_first, o_wide = _oracle(first, xs), _oracle(wide, xs)
    with Engine(0) as eng:
        a = fit(first, eng)
        b = fit(wide, eng)
        b2 = fit(wide, eng)
        knob.setenv("LFE_SUMS_CG", "0")
        b_flat = fit(wide, eng)
    _check(a, o_first)
    _check(b, o_wide)
    _check(b_flat, o_wide)
    np.testing.assert_array_equal(b[0], b2[0])
    np.testing.assert_array_equal(b[1], b2[1])
    np.testing.assert_allclose(b[0], b_flat[0], rtol=1e-12, atol=0)
