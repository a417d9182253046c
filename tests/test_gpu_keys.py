"""Host prep on the device: integer id factorization and the
exact distinct-row count behind estimate_compression_ratio (compress.py:187-253).
References: np.unique (sorted-unique codes, as polars_impl.py:118-139 needs only
group membership) and a host count over canonicalized row bytes."""
from __future__ import annotations

import os

import numpy as np
import pytest

from leanfe_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from leanfe_amd._lib import Engine
    with Engine(0) as e:
        yield e


@pytest.mark.parametrize("case", ["random", "negative_wide", "extremes", "constant", "single"])
def test_factorize_ids_matches_np_unique(eng, case):
    rng = np.random.default_rng(5)
    if case == "random":
        ids = rng.integers(0, 10**12, 1_000_003)
        ids[::7] = ids[3]  # duplicates
    elif case == "negative_wide":
        ids = rng.integers(-(2**62), 2**62, 300_000)
        ids[100:5000] = ids[:4900]
    elif case == "extremes":
        ids = np.array([np.iinfo(np.int64).max, np.iinfo(np.int64).min, 0, -1, 1, np.iinfo(np.int64).max] * 1000)
    elif case == "constant":
        ids = np.full(70_000, 123456789012)
    else:
        ids = np.array([42])
    codes, G = eng.factorize_ids(ids)
    uniq, inv = np.unique(ids, return_inverse=True)
    assert G == uniq.size
    np.testing.assert_array_equal(codes, inv.ravel())


def _host_distinct(cols, codes):
    canon = []
    for c in cols:
        v = np.asarray(c, dtype=np.float64).copy()
        v[v == 0.0] = 0.0
        bits = v.view(np.uint64).copy()
        bits[np.isnan(v)] = np.uint64(0x7FF8000000000000)
        canon.append(bits)
    for k in codes:
        canon.append(np.asarray(k, dtype=np.uint64))
    return np.unique(np.stack(canon, axis=1), axis=0).shape[0]


@pytest.mark.parametrize("hash_bits", [64, 10])
def test_count_distinct_rows_exact(eng, hash_bits, knob):
    rng = np.random.default_rng(9)
    n = 400_000
    y = rng.standard_normal(n)                     # y is not part of the key
    x1 = rng.integers(0, 3, n).astype(np.float64)
    x2 = rng.choice(np.array([-0.0, 0.0, 1.5, np.nan, -np.nan]), n)
    x3 = np.where(rng.random(n) < 0.5, 2.0, rng.integers(0, 50, n).astype(np.float64))
    fe1 = rng.integers(0, 40, n).astype(np.int32)
    fe2 = rng.integers(0, 7, n).astype(np.int32)
    eng.load([y, x1, x2, x3], [fe1, fe2], [40, 7])
    knob.setenv("LFE_ROW_HASH_BITS", str(hash_bits))  # 10 bits: thousands of collisions -> exact recount
    try:
        got = eng.count_distinct_rows()
    finally:
        knob.delenv("LFE_ROW_HASH_BITS")
    assert got == _host_distinct([x1, x2, x3], [fe1, fe2])


def test_auto_strategy_ratio_and_device_factorized_ids():
    """strategy='auto' reports the exact ratio; sparse int64 FE ids (factorized on the
    device) give the same fit as their dense codes."""
    from leanfe_amd import leanfe_hip
    from leanfe_amd.strategy import estimate_compression_ratio
    n, L = 120_000, [3000, 40]
    data = synth.panel(n, 2, L, seed=17)
    data["x1"] = np.round(data["x1"], 1)  # some repeated rows
    ref = leanfe_hip(data, formula="y ~ x1 + x2 | fe1 + fe2", vcov="HC1", quiet=True)
    sparse = dict(data)
    sparse["fe1"] = data["fe1"].astype(np.int64) * 1_000_003_000_017 - 5  # ids far beyond 4n
    r = leanfe_hip(sparse, formula="y ~ x1 + x2 | fe1 + fe2", vcov="HC1", quiet=True)
    assert r.compression_ratio == pytest.approx(estimate_compression_ratio(
        [data["x1"], data["x2"], data["fe1"], data["fe2"]]), rel=0, abs=0)
    assert r.fe_dims == ref.fe_dims and r.iterations == ref.iterations and r.n_obs == ref.n_obs
    for x in ("x1", "x2"):
        assert r.coefs[x] == pytest.approx(ref.coefs[x], rel=1e-12)
        assert r.std_errors[x] == pytest.approx(ref.std_errors[x], rel=1e-12)


@pytest.mark.parametrize("case", ["floats", "floats_nan_signed_zero"])
def test_factorize_float_ids_match_np_unique(eng, case):
    """Float FE / cluster ids go through the device sort via order-preserving int64 keys
    (frame.float_order_keys): codes equal np.unique's inverse."""
    from leanfe_amd import frame
    rng = np.random.default_rng(5)
    v = rng.normal(size=300_000) * 1e6
    v = np.round(v[rng.integers(0, 40_000, v.size)], 3)
    if case == "floats_nan_signed_zero":
        v[::97] = np.nan
        v[::89] = 0.0
        v[::83] = -0.0
        v[::79] = -np.inf
    codes, G = frame.factorize(v, device=eng)
    uniq, inv = np.unique(v, return_inverse=True)
    assert G == uniq.size
    np.testing.assert_array_equal(codes, inv.ravel())


def test_sparse_cluster_ids_factorized_on_device_same_fit():
    """Sparse int64 / float cluster ids (factorized on the device, hip_impl._cluster_se) give
    the same two-way clustered fit as their dense codes (std_errors.py:354-441)."""
    from leanfe_amd import leanfe_hip
    n, L = 150_000, [2000, 60, 300]
    data = synth.panel(n, 3, L, seed=23)
    ref = leanfe_hip(data, formula="y ~ x1 + x2 + x3 | fe1 + fe2", vcov="cluster",
                     cluster_cols=["fe2", "fe3"], quiet=True)
    sparse = dict(data)
    sparse["fe3"] = data["fe3"].astype(np.int64) * 7_000_000_000_019 + 11
    sparse["fe2"] = data["fe2"].astype(np.float64) * 0.37 - 5.0
    r = leanfe_hip(sparse, formula="y ~ x1 + x2 + x3 | fe1 + fe2", vcov="cluster",
                   cluster_cols=["fe2", "fe3"], quiet=True)
    assert r.n_clusters == ref.n_clusters and r.n_obs == ref.n_obs and r.iterations == ref.iterations
    for x in ("x1", "x2", "x3"):
        assert r.coefs[x] == pytest.approx(ref.coefs[x], rel=1e-12)
        assert r.std_errors[x] == pytest.approx(ref.std_errors[x], rel=1e-12)


def _same_partition(codes, G, ref_inv, ref_G):
    """codes and ref_inv group the rows identically (codes may be numbered differently)."""
    assert G == ref_G
    assert codes.min() >= 0 and codes.max() == G - 1
    # a bijection between the two labelings: each code maps to exactly one reference code
    pairs = np.unique(np.stack([codes.astype(np.int64), ref_inv.astype(np.int64)], axis=1), axis=0)
    assert pairs.shape[0] == G


def _words(rng, n, n_distinct):
    alphabet = np.array(list("abcxyzÆøå中文 _-0123456789"))
    pool = ["".join(rng.choice(alphabet, rng.integers(0, 24))) for _ in range(n_distinct)]
    pool[0] = ""  # the empty string is a value of its own
    pool[1] = "a" * 40  # long, shares a prefix with pool[2]
    pool[2] = "a" * 39 + "b"
    pool = list(dict.fromkeys(pool))
    return np.array(pool, dtype=object)[rng.integers(0, len(pool), n)]


@pytest.mark.parametrize("hash_bits", [64, 8])
def test_factorize_strings_exact_grouping(eng, hash_bits, knob):
    """String FE ids (_cats_to_int's String -> Categorical cast, polars_impl.py:118-139) are
    grouped on the device exactly as np.unique groups them; 8-bit hashes force thousands of
    collisions through the exact split (k_str_exact)."""
    from leanfe_amd import frame
    rng = np.random.default_rng(31)
    v = _words(rng, 200_000 if hash_bits == 64 else 30_000, 3000)
    knob.setenv("LFE_STR_HASH_BITS", str(hash_bits))
    try:
        codes, G = frame.factorize(v, device=eng)
    finally:
        knob.delenv("LFE_STR_HASH_BITS")
    uniq, inv = np.unique(v.astype(str), return_inverse=True)
    _same_partition(codes, G, inv.ravel(), uniq.size)


def test_factorize_strings_frequent_value_beside_collisions(eng, knob):
    """A very frequent string whose hash run holds only that string is not walked by the exact
    split, even when other runs collide (20-bit hashes over 20K strings: ~200 colliding pairs);
    the grouping is exact (k_str_exact walked every run head serially)."""
    import time

    from leanfe_amd import frame
    rng = np.random.default_rng(5)
    pool = _words(rng, 20_000, 20_000)
    v = np.concatenate([np.array(["the frequent value"] * 1_000_000, dtype=object), pool[rng.integers(0, pool.size, 500_000)]])
    v = v[rng.permutation(v.size)]
    knob.setenv("LFE_STR_HASH_BITS", "20")
    try:
        t0 = time.perf_counter()
        codes, G = frame.factorize(v, device=eng)
        dt = time.perf_counter() - t0
    finally:
        knob.delenv("LFE_STR_HASH_BITS")
    uniq, inv = np.unique(v.astype(str), return_inverse=True)
    _same_partition(codes, G, inv.ravel(), uniq.size)
    assert dt < 10.0, dt


@pytest.mark.parametrize("case", ["single", "all_equal", "all_empty", "bytes", "arrow_slice"])
def test_factorize_strings_edge_cases(eng, case):
    import pyarrow as pa
    from leanfe_amd import frame
    if case == "single":
        v, ref = np.array(["only"]), np.array(["only"])
    elif case == "all_equal":
        v = ref = np.array(["same"] * 5000, dtype=object)
    elif case == "all_empty":
        v = ref = np.array([""] * 777, dtype=object)
    elif case == "bytes":
        v = ref = np.array([b"\x00", b"", b"\x00\x00", b"\x00", b"ab"] * 300, dtype=object)
    else:
        full = pa.array(["p", "q", "p", "r", "q", "p", "s"] * 200)
        v = full.slice(3, 1000)
        ref = np.array(v.to_pylist(), dtype=object)
    codes, G = frame.factorize(v, device=eng)
    uniq, inv = np.unique(ref, return_inverse=True)
    _same_partition(codes, G, inv.ravel(), uniq.size)


def test_string_fe_columns_same_fit():
    """A fit with string FE and cluster columns (factorized on the device) equals the fit on
    their integer codes (β / SE within 1e-12, integers equal)."""
    from leanfe_amd import leanfe_hip
    n, L = 150_000, [2000, 60, 300]
    data = synth.panel(n, 3, L, seed=29)
    ref = leanfe_hip(data, formula="y ~ x1 + x2 + x3 | fe1 + fe2", vcov="cluster",
                     cluster_cols=["fe3"], quiet=True)
    s = dict(data)
    s["fe1"] = np.array([f"firm-{g:05d}" for g in data["fe1"]], dtype=object)
    s["fe2"] = np.array([f"yr{g}" for g in data["fe2"]], dtype=object)
    s["fe3"] = np.array([f"state_{g}" for g in data["fe3"]], dtype=object)
    r = leanfe_hip(s, formula="y ~ x1 + x2 + x3 | fe1 + fe2", vcov="cluster", cluster_cols=["fe3"], quiet=True)
    assert r.n_clusters == ref.n_clusters and r.n_obs == ref.n_obs and r.iterations == ref.iterations
    assert sorted(r.fe_dims) == sorted(ref.fe_dims)
    for x in ("x1", "x2", "x3"):
        assert r.coefs[x] == pytest.approx(ref.coefs[x], rel=1e-12)
        assert r.std_errors[x] == pytest.approx(ref.std_errors[x], rel=1e-12)
