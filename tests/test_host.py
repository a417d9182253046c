"""CPU: host-side logic of the hip backend (no GPU calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

from leanfe_amd import frame, inference, synth
from leanfe_amd.formula import parse_formula
from leanfe_amd.result import LeanFEResult
from leanfe_amd.strategy import determine_strategy, estimate_compression_ratio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---------------------------------------------------------------- formula
# cases mirror the grammar of common.py:51-181


def test_formula_basic():
    f = parse_formula("y ~ x1 + x2 | fe1 + fe2")
    assert f.y_col == "y" and f.x_cols == ["x1", "x2"] and f.fe_cols == ["fe1", "fe2"]
    assert f.factor_vars == [] and f.interactions == [] and f.instruments == []


def test_formula_no_fe_and_iv():
    assert parse_formula("y ~ x").fe_cols == []
    f = parse_formula("y ~ x1 | fe | z1 + z2")
    assert f.instruments == ["z1", "z2"]


def test_formula_factor_and_interaction():
    f = parse_formula("y ~ x + i(region, ref=R1) + treat:i(region) + i(year) | fe")
    assert f.x_cols == ["x"]
    assert f.factor_vars == [("region", "R1"), ("year", None)]
    assert f.interactions == [("treat", "region", None)]
    f = parse_formula('y ~ treat:i(region, ref="R2") | fe')
    assert f.interactions == [("treat", "region", "R2")]


def test_formula_errors():
    with pytest.raises(ValueError):
        parse_formula("y ~ x | a | b | c")
    with pytest.raises(ValueError):
        parse_formula("y x")
    with pytest.raises(ValueError):
        parse_formula("y ~ i(1bad-) | fe")


# ---------------------------------------------------------------- result


def test_result_dict_interface_and_pvalues():
    r = LeanFEResult(coefs={"x": 2.0, "z": 0.0}, std_errors={"x": 0.5, "z": 0.0}, n_obs=1000,
                     vcov_type="iid", df_resid=990, iterations=4, fe_cols=["a", "b"], fe_dims=(10, 5))
    assert r["coefs"]["x"] == 2.0 and r["iterations"] == 4
    assert repr(r["n_obs"]) == "1_000"
    from scipy import stats
    assert np.isclose(r.p_values["x"], 2 * (1 - stats.t.cdf(4.0, 990)))
    assert np.isnan(r.t_stats["z"])
    lo, hi = r.confint()["x"]
    assert lo < 2.0 < hi
    s = str(r)
    assert "FE Dimensions: 10 × 5" in s and "Variable" in s
    assert set(r.keys()) >= {"coefs", "std_errors", "n_obs", "iterations", "df_resid", "n_clusters"}


# ---------------------------------------------------------------- strategy (compress.py:96-184)


def test_determine_strategy_rules():
    assert determine_strategy("iid", True, {"a": 5}) == "alt_proj"
    assert determine_strategy("iid", False, {"a": 10_001, "b": 3}) == "alt_proj"
    assert determine_strategy("iid", False, {"a": 9_000, "b": 12_000}) == "alt_proj"
    assert determine_strategy("iid", False, {"a": 50, "b": 20}) == "compress"
    assert determine_strategy("iid", False, {"a": 5000, "b": 5000}, n_obs=1000,
                              estimated_compression_ratio=1.0) == "alt_proj"
    assert determine_strategy("weird", False, {"a": 5}) == "alt_proj"


def test_compression_ratio_exact_small():
    x = np.array([1, 1, 2, 2, 2.0])
    fe = np.array([1, 1, 2, 3, 3])
    assert estimate_compression_ratio([x, fe]) == pytest.approx(3 / 5)


# ---------------------------------------------------------------- frame


def test_factorize_fast_path_and_unique():
    c, g = frame.factorize(np.array([3, 0, 3, 7]))
    assert c.dtype == np.int32 and g == 8 and c.tolist() == [3, 0, 3, 7]
    c, g = frame.factorize(np.array(["b", "a", "b"]))
    assert g == 2 and c.tolist() == [1, 0, 1]
    c, g = frame.factorize(np.array([-5, 10, -5]))
    assert g == 2 and c.tolist() == [0, 1, 0]


def test_string_buffers_arrow_layout():
    """The host hand-off of lfe_factorize_strings: int64 offsets from 0 and the bytes; None
    for nulls and mixed types (those keep the host's sorted unique)."""
    import pyarrow as pa
    off, data = frame.string_buffers(np.array(["ab", "", "héllo"], dtype=object))
    assert off.tolist() == [0, 2, 2, 8] and bytes(data) == "abhéllo".encode()
    off, data = frame.string_buffers(pa.array(["q", "rr", "s"]).slice(1))
    assert off.tolist() == [0, 2, 3] and bytes(data) == b"rrs"
    off, data = frame.string_buffers(np.array([b"\x00a", b"z"], dtype=object))
    assert off.tolist() == [0, 2, 3] and bytes(data) == b"\x00az"
    assert frame.string_buffers(np.array(["x", None], dtype=object)) is None
    assert frame.string_buffers(np.array([1, "a"], dtype=object)) is None
    assert frame.string_buffers(np.array([1.5, 2.5])) is None


def test_intersect_membership():
    a = np.array([0, 0, 1, 1, 0], dtype=np.int32)
    b = np.array([0, 1, 0, 1, 0], dtype=np.int32)
    c, g = frame.intersect([a, b], [2, 2])
    assert c[0] == c[4] and len(set(c.tolist())) == 4 and g >= 4


def test_expand_factors_and_interactions():
    cols = {"r": np.array(["A", "B", "C", "A"]), "t": np.array([1.0, 2.0, 3.0, 4.0])}
    names = frame.expand_factors(cols, [("r", None)])
    assert names == ["r_B", "r_C"] and cols["r_B"].tolist() == [0, 1, 0, 0]
    names = frame.expand_interactions(cols, [("t", "r", "B")])
    assert names == ["t_A", "t_C"] and cols["t_C"].tolist() == [0, 0, 3.0, 0]
    with pytest.raises(ValueError):
        frame.expand_factors(cols, [("r", "Z")])


def test_get_columns_pandas_and_dict():
    import pandas as pd
    df = pd.DataFrame({"a": [1.0, 2.0], "c": pd.Categorical(["x", "y"])})
    out = frame.get_columns(df, ["a", "c"])
    assert out["c"].tolist() == [0, 1]
    with pytest.raises(ValueError):
        frame.get_columns({"a": [1]}, ["a", "b"])


# ---------------------------------------------------------------- inference


def test_split_gram_and_solve():
    rng = np.random.default_rng(0)
    X = np.column_stack([np.ones(50), rng.normal(size=(50, 3))])
    y = X @ np.array([1.0, 2.0, -1.0, 0.5]) + rng.normal(size=50) * 0.1
    Z = np.column_stack([np.ones(50), y, X[:, 1:]])
    XtX, Xty = inference.split_gram(Z.T @ Z)
    b, inv = inference.solve_normal(XtX, Xty)
    np.testing.assert_allclose(b, np.linalg.lstsq(X, y, rcond=None)[0], rtol=1e-10)
    np.testing.assert_allclose(inv @ XtX, np.eye(4), atol=1e-10)


def test_multiway_subsets_order():
    assert inference.cluster_subsets(3) == [(0,), (1,), (2,), (0, 1), (0, 2), (1, 2), (0, 1, 2)]


# ---------------------------------------------------------------- synthetic panel


def test_synth_counter_based_and_shardable():
    full = synth.panel(1000, 3, [50, 7], seed=12345)
    part = synth.panel(400, 3, [50, 7], seed=12345, row_offset=600)
    for k in full:
        np.testing.assert_array_equal(full[k][600:], part[k])
    assert full["fe1"].max() < 50 and full["fe2"].min() >= 0
    assert abs(float(np.mean(synth.normal(np.arange(20000, dtype=np.uint64), 5, 1)))) < 0.05


# ---------------------------------------------------------------- C ABI surface


def _declared_symbols():
    txt = open(os.path.join(ROOT, "include", "leanfe_hip.h")).read()
    return sorted(set(re.findall(r"\b(lfe_[a-z_0-9]+)\s*\(", txt)))


def test_header_matches_binding_table():
    from leanfe_amd._lib import SIGNATURES
    assert sorted(SIGNATURES) == _declared_symbols()


def test_library_loads_and_exports_every_symbol():
    path = os.path.join(ROOT, "leanfe_amd", "liblfe_hip.so")
    if not os.path.exists(path):
        from leanfe_amd.build import build
        build(verbose=False)
    lib = ctypes.CDLL(path)
    for name in _declared_symbols():
        assert hasattr(lib, name), name
    lib.lfe_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.lfe_version()


def test_library_is_built_from_the_checked_out_sources(tmp_path):
    """build.py stamps the hash of every engine source into the library (lfe_build_hash) and the
    loader refuses a library whose stamp differs, so a stale build cannot run silently."""
    from leanfe_amd import build as B
    from leanfe_amd import _lib

    B.build(verbose=False)  # content-hash incremental: a no-op when the library is current
    lib = ctypes.CDLL(B.LIB)
    lib.lfe_build_hash.restype = ctypes.c_char_p
    assert lib.lfe_build_hash().decode() == B.source_hash() == B.library_hash()
    stale = tmp_path / "liblfe_hip.so"
    stale.write_bytes(open(B.LIB, "rb").read().replace(B.source_hash().encode(), b"0" * 32))
    assert B.library_hash(str(stale)) == "0" * 32
    old = _lib.LIB_PATH
    try:  # the loader's check, pointed at the stale copy
        _lib.LIB_PATH = str(stale)
        saved, _lib._lib = _lib._lib, None
        with pytest.raises(ImportError, match="other sources"):
            _lib.load_library()
    finally:
        _lib.LIB_PATH = old
        _lib._lib = saved


@pytest.mark.parametrize("weighted,z_ones", [(False, False), (True, False), (False, True)])
def test_iv_system_matches_oracle_2sls(weighted, z_ones):
    """inference.IVSystem (2SLS from the (p+1)^2 Gram of [1, y, x, z] plus the u-space
    meat transform) == the oracle's restatement of polars_impl.py:176-198 +
    common.py:188-287 + std_errors.py:448-470 on the same columns."""
    from leanfe_amd import inference
    from oracle import altproj
    rng = np.random.default_rng(5)
    n, k, m = 4000, 2, 2
    X = rng.normal(size=(n, k))
    Z = np.column_stack([X[:, 1], rng.normal(size=n) + 0.5 * X[:, 0]])
    if z_ones:
        Z = np.column_stack([np.ones(n), Z])
        m = 3
    y = X @ np.array([1.0, -0.5]) + rng.normal(size=n)
    w = rng.uniform(0.5, 2.0, n) if weighted else None
    o = altproj.run_regression_iv(y, X, Z, w, "HC1", None, True, n, 0)
    D = np.column_stack([np.ones(n), y, X, Z])
    Dw = D * np.sqrt(w)[:, None] if weighted else D
    iv = inference.IVSystem(Dw.T @ Dw, k, m, z_has_ones=z_ones)
    np.testing.assert_allclose(iv.beta_full, o["beta_full"], rtol=1e-12)
    np.testing.assert_allclose(iv.XtX_inv, o["XtX_inv"], rtol=1e-10)
    u = np.column_stack([np.ones(n), X, Z])
    r = y - u @ iv.coef
    np.testing.assert_allclose(r, o["resid"], rtol=1e-10, atol=1e-12)
    s = r ** 2 * (w if weighted else 1.0)
    meat_u = u.T @ (u * s[:, None])
    se = inference.se_hc1(iv.XtX_inv, iv.xhat_meat(meat_u), n, n - (k + 1))
    np.testing.assert_allclose(se[1:], o["se"], rtol=1e-10)


def test_stream_parquet_batches_cover_rows_in_order(tmp_path):
    """frame.stream_parquet (the streaming ingest of a Parquet path) yields every row once,
    in file order, with the requested columns only."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    n = 10_007
    d = {"y": np.arange(n, dtype=np.float64), "x": np.arange(n, dtype=np.float64) * 2, "fe": np.arange(n) % 7}
    path = str(tmp_path / "p.parquet")
    pq.write_table(pa.table(d), path, row_group_size=3000)
    assert frame.parquet_rows(path) == n
    seen = []
    for row0, b in frame.stream_parquet(path, ["y", "x"], batch_rows=1024):
        assert set(b) == {"y", "x"}
        assert b["y"][0] == row0 and np.array_equal(b["x"], 2 * b["y"])
        seen.append((row0, len(b["y"])))
    assert seen[0][0] == 0 and sum(m for _, m in seen) == n
    assert all(r + m == r2 for (r, m), (r2, _) in zip(seen, seen[1:]))


def test_float_order_keys_preserve_np_unique_order():
    """The int64 keys behind device-factorized float ids sort like np.unique sorts the floats
    (-0.0 == 0.0, NaNs last and alike), so sorted-unique codes agree."""
    from leanfe_amd.frame import float_order_keys
    v = np.array([3.5, -0.0, 0.0, np.nan, -np.inf, np.inf, -2.25, 1e-300, -1e-300, np.nan, 3.5, -7e10])
    k = float_order_keys(v)
    uk, ik = np.unique(k, return_inverse=True)
    uv, iv = np.unique(v, return_inverse=True)
    assert uk.size == uv.size
    np.testing.assert_array_equal(ik.ravel(), iv.ravel())


# ---------------------------------------------------------------- stream discipline (source check)
# Round 4 found a race in the emulated collectives: a null-stream hipMemcpy is not ordered against
# a context's non-blocking stream, so a kernel read an all-to-all block before it landed.
# Every device copy, fill, kernel launch and RCCL call of the engine therefore goes on the context's
# own stream (the work-item upload on its side stream, joined by events); synchronous null-stream
# copies are allowed only in the opt-in timing diagnostics that read their stamps after a sync.

_STREAM_CALLS = re.compile(r"\b(hipMemcpyAsync|hipMemsetAsync|hipMemcpy|hipMemset|hipLaunchKernelGGL|hipLaunchKernel|"
                           r"ncclAllReduce|ncclSend|ncclRecv|ncclBroadcast|ncclAllGather|ncclReduceScatter)\s*\(")
_DIAG_SYNC_OK = {"lfe_dense.hip": 5, "lfe_iter.hip": 1}  # LFE_DN8_TIMING / LFE_SWEEP_TIMING stamps


def _call_args(src, i):
    depth, cur, out = 0, "", []
    for ch in src[i:]:
        if ch == "(":
            depth += 1
            if depth == 1:
                continue
        elif ch == ")":
            depth -= 1
            if depth == 0:
                out.append(cur.strip())
                return out
        if ch == "," and depth == 1:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    raise AssertionError("unbalanced call")


def test_every_device_operation_is_issued_on_the_context_stream():
    import glob

    sync_calls = {}
    checked = 0
    for path in sorted(glob.glob(os.path.join(ROOT, "leanfe_amd", "csrc", "*.hip"))):
        src = open(path).read()
        name = os.path.basename(path)
        for m in _STREAM_CALLS.finditer(src):
            fn = m.group(1)
            args = _call_args(src, m.end() - 1)
            line = src.count("\n", 0, m.start()) + 1
            if fn in ("hipMemcpy", "hipMemset"):
                sync_calls[name] = sync_calls.get(name, 0) + 1
                continue
            stream = args[4] if fn == "hipLaunchKernelGGL" else args[-1]
            if fn == "hipLaunchKernelGGL" and stream == "s":  # the one helper that takes its stream
                continue
            ok = {"c->stream"} | ({"c->up_stream"} if fn == "hipMemcpyAsync" else set())
            assert stream in ok, f"{name}:{line}: {fn} on '{stream}', not the context stream"
            checked += 1
    assert checked > 250
    assert sync_calls == _DIAG_SYNC_OK, sync_calls


def test_expansion_plan_applied_per_chunk_equals_whole_columns():
    """frame.Expansion (the out-of-core path's lazy i(var) / var:i(f) expansion): the columns it
    forms chunk by chunk are the whole-column expansion (polars_impl.py:27-115), names and order
    included, for string and integer factors and a chosen reference category."""
    rng = np.random.default_rng(3)
    n = 10_007
    cols = {"year": rng.integers(2000, 2012, n), "region": rng.choice(np.array(["N", "S", "E", "W"]), n),
            "treat": rng.standard_normal(n)}
    inter, facs = [("treat", "region", "S")], [("year", 2005)]
    whole = dict(cols)
    names = frame.expand_interactions(whole, inter) + frame.expand_factors(whole, facs)
    plan = frame.Expansion(cols, inter, facs)
    assert plan.names == names and plan.numeric_sources == ["treat"]
    assert "region_S" not in [nm.split("treat_")[-1] for nm in names] and "year_2005" not in names
    for r0 in range(0, n, 3_000):
        sl = slice(r0, min(n, r0 + 3_000))
        chunk = plan.columns(cols, {"treat": cols["treat"][sl]}, sl)
        for name, col in zip(names, chunk):
            np.testing.assert_array_equal(col, whole[name][sl])


def test_int_range_matches_numpy():
    """lfe_int_range (frame.factorize's dense-code test on host threads) = NumPy's min / max for
    every signed width, extremes and odd lengths included (host code: no GPU)."""
    from leanfe_amd import frame
    from leanfe_amd._lib import int_range

    rng = np.random.default_rng(5)
    for dt in (np.int8, np.int16, np.int32, np.int64):
        info = np.iinfo(dt)
        for n in (1, 7, 1_000_003, 5_000_001):
            v = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
            assert int_range(v) == (int(v.min()), int(v.max()))
        v = np.zeros(4_200_000, dtype=dt)
        v[-1], v[0] = info.max, info.min
        assert int_range(v) == (int(info.min), int(info.max)) == frame.int_range(v)
