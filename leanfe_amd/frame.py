"""Host-side data preparation for the HIP backend.

Replaces the Polars data handling in front of the reference's hot path:
column selection (polars_impl.py:324-347), categorical -> integer codes
(``_cats_to_int``, :118-139), factor/interaction expansion (:27-115) and the
hand-off of NumPy columns to the engine.  Accepted inputs: a mapping of
array-likes, a pandas DataFrame, a pyarrow Table, a Parquet path, or a Polars
DataFrame/LazyFrame when ``polars`` is importable.
"""
from __future__ import annotations

from collections.abc import Mapping

import numpy as np


def get_columns(data, names: list[str]) -> dict[str, np.ndarray]:
    names = list(dict.fromkeys(names))
    if isinstance(data, str):
        import pyarrow.parquet as pq
        t = pq.read_table(data, columns=names)
        return {c: _arrow_to_numpy(t.column(c)) for c in names}
    mod = type(data).__module__
    if mod.startswith("polars"):
        df = data.select(names)
        if hasattr(df, "collect"):
            df = df.collect()
        return {c: _polars_to_numpy(df[c]) for c in names}
    if mod.startswith("pyarrow"):
        return {c: _arrow_to_numpy(data.column(c)) for c in names}
    if mod.startswith("pandas"):
        out = {}
        for c in names:
            s = data[c]
            if str(s.dtype) == "category":
                out[c] = np.asarray(s.cat.codes.to_numpy(), dtype=np.int64)
            else:
                out[c] = s.to_numpy()
        return out
    if isinstance(data, Mapping) or hasattr(data, "__getitem__"):
        missing = [c for c in names if c not in data]
        if missing:
            raise ValueError(f"columns not found in data: {missing}")
        return {c: np.asarray(data[c]) for c in names}
    raise TypeError(f"unsupported data type: {type(data)!r}")


def parquet_rows(path: str) -> int:
    import pyarrow.parquet as pq
    return int(pq.ParquetFile(path).metadata.num_rows)


def stream_parquet(path: str, names: list[str], batch_rows: int = 1 << 22, row_range=None):
    """Yield (row0, {name: ndarray}) batches of a Parquet file's columns, in file order
    (the streaming counterpart of ``pl.scan_parquet``, polars_impl.py:341-343): one
    batch is decoded while the previous one is uploaded.  ``row_range`` (lo, hi): only
    those rows, from the row groups that hold them, with row0 counted from lo."""
    import pyarrow.parquet as pq
    pf = pq.ParquetFile(path)
    groups, skip, lo, hi = None, 0, 0, None
    if row_range is not None:
        lo, hi = (int(x) for x in row_range)
        groups, start = [], 0
        for g in range(pf.metadata.num_row_groups):
            end = start + pf.metadata.row_group(g).num_rows
            if end > lo and start < hi:
                if not groups:
                    skip = lo - start
                groups.append(g)
            start = end
    row0 = 0
    for rb in pf.iter_batches(batch_size=int(batch_rows), columns=list(names), row_groups=groups):
        a, b = 0, rb.num_rows
        if row_range is not None:
            a = min(skip, b)
            skip -= a
            b = min(b, a + (hi - lo) - row0)
            if b <= a:
                if row0 >= hi - lo:
                    break
                continue
        out = {c: _arrow_to_numpy(rb.column(c).slice(a, b - a)) for c in names}
        yield row0, out
        row0 += b - a


def _arrow_to_numpy(col) -> np.ndarray:
    import pyarrow as pa
    if pa.types.is_dictionary(col.type):
        col = col.combine_chunks()
        return np.asarray(col.indices.to_numpy(zero_copy_only=False), dtype=np.int64)
    return col.to_numpy()


def _polars_to_numpy(s) -> np.ndarray:
    if str(s.dtype) in ("Categorical", "Enum"):
        return s.to_physical().to_numpy()
    return s.to_numpy()


def int_range(v: np.ndarray) -> tuple[int, int]:
    """(min, max) of an integer array: past 4M signed values one pass over host threads in the
    engine library (lfe_int_range: NumPy's two single-threaded reductions took 14 ms per 50M-row
    code column of a 146 ms end-to-end fit, profiles/r06/e2e_profile.txt)."""
    if v.size >= (1 << 22) and v.dtype.kind == "i":
        try:
            from leanfe_amd._lib import int_range as lib_range
            return lib_range(v)
        except OSError:  # the library is not built (host-only use): NumPy
            pass
    return int(v.min()), int(v.max())


def factorize(values, global_codes: bool = False, device=None) -> tuple[np.ndarray, int]:
    """Dense int32 group codes and the number of code values.

    Non-negative integer columns whose maximum is below max(4n, 2^20) are used
    as codes directly (O(n); unused code values are empty groups, which every
    kernel ignores).  Without ``device`` anything else (strings, floats, sparse
    ids) goes through a sorted unique.  Only group membership matters for the
    estimator: the codes' numbering is not part of the result.

    ``global_codes`` (row shards of one fit): the values must already be global
    non-negative integer codes and are used as they are, since a per-shard
    unique would number the groups differently on every rank.

    ``device`` (an ``Engine``): sparse integer and float ids are factorized on the GPU
    (``Engine.factorize_ids``, a radix sort; same codes as the sorted unique); strings and
    bytes without nulls too (``Engine.factorize_strings``), whose codes follow the order of
    the strings' 64-bit hashes, not lexicographic order (same groups as the sorted unique).
    String columns with nulls, or without pyarrow, keep the sorted unique."""
    v = np.asarray(values)
    n = v.size
    if global_codes:
        if n == 0:
            return np.zeros(0, dtype=np.int32), 1
        if not (np.issubdtype(v.dtype, np.integer) or v.dtype == np.bool_):
            raise ValueError("sharded fits need global non-negative integer FE / cluster codes")
        vmin, vmax = int_range(v)
        if vmin < 0 or vmax >= 2 ** 31 - 1:
            raise ValueError("sharded fits need global integer codes in [0, 2^31 - 1)")
        return v.astype(np.int32, copy=False), vmax + 1
    if n == 0:
        return np.zeros(0, dtype=np.int32), 1
    if np.issubdtype(v.dtype, np.integer) or v.dtype == np.bool_:
        vmin, vmax = int_range(v) if v.dtype != np.bool_ else (int(v.min()), int(v.max()))
        if vmin >= 0 and vmax < max(4 * n, 1 << 20) and vmax < 2 ** 31 - 1:
            return v.astype(np.int32, copy=False), vmax + 1
        if device is not None and n < 2 ** 31 - 1 and (v.dtype != np.uint64 or vmax < 2 ** 63):
            return device.factorize_ids(v.astype(np.int64, copy=False))
    elif device is not None and n < 2 ** 31 - 1 and v.dtype in (np.float64, np.float32):
        return device.factorize_ids(float_order_keys(v))
    elif device is not None and n < 2 ** 31 - 1 and v.dtype.kind in ("U", "S", "O"):
        sb = string_buffers(v)
        if sb is not None:  # strings without nulls: grouped on the device (_cats_to_int's String cast)
            return device.factorize_strings(*sb)
    uniq, inv = np.unique(v, return_inverse=True)
    return inv.astype(np.int32).ravel(), int(uniq.size)


def string_buffers(values) -> tuple[np.ndarray, np.ndarray] | None:
    """Arrow layout of a string (or bytes) column: int64 offsets [n + 1] starting at 0 and the
    uint8 bytes, for ``lfe_factorize_strings``.  None when the values are not all strings / all
    bytes or hold nulls (those keep the host's sorted unique), and None without pyarrow."""
    try:
        import pyarrow as pa
    except ImportError:
        return None

    if isinstance(values, pa.ChunkedArray):
        arr = values.combine_chunks()
    elif isinstance(values, pa.Array):
        arr = values
    else:
        v = np.asarray(values)
        kinds = {"U": [pa.large_string()], "S": [pa.large_binary()], "O": [pa.large_string(), pa.large_binary()]}
        arr = None
        for t in kinds.get(v.dtype.kind, []):
            try:
                arr = pa.array(v, type=t, from_pandas=False)
                break
            except (pa.ArrowInvalid, pa.ArrowTypeError, TypeError):
                continue
        if arr is None:
            return None
    if arr.null_count:
        return None
    if pa.types.is_string(arr.type) or pa.types.is_large_string(arr.type):
        arr = arr.cast(pa.large_string())
    elif pa.types.is_binary(arr.type) or pa.types.is_large_binary(arr.type):
        arr = arr.cast(pa.large_binary())
    else:
        return None
    bufs = arr.buffers()
    off = np.frombuffer(bufs[1], dtype=np.int64, count=len(arr) + 1, offset=arr.offset * 8)
    data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, np.uint8)
    lo, hi = int(off[0]), int(off[-1])
    return off - lo, data[lo:hi]


def float_order_keys(v: np.ndarray) -> np.ndarray:
    """int64 keys whose signed order is the float order of ``v`` (np.unique's): -0.0 and 0.0 map
    to one key, every NaN to one key above +inf; so the device's sorted-unique codes of the
    keys are np.unique's codes of the floats."""
    f = np.ascontiguousarray(v, dtype=np.float64)
    f = np.where(f == 0.0, 0.0, f)  # -0.0 -> +0.0
    b = f.view(np.int64).copy()
    b[np.isnan(f)] = 0x7FF8000000000000
    neg = b < 0
    b[neg] ^= np.int64(0x7FFFFFFFFFFFFFFF)
    return b


def intersect(codes: list[np.ndarray], levels: list[int]) -> tuple[np.ndarray, int]:
    """Composite-key codes for ``group_by([c1, c2, ...])`` (std_errors.py:399-408)."""
    if len(codes) == 1:
        return codes[0], levels[0]
    key = codes[0].astype(np.int64)
    span = levels[0]
    for c, g in zip(codes[1:], levels[1:]):
        if span * g < 2 ** 62:
            key = key * g + c
            span = span * g
        else:
            key, span = _dense(key)
            key = key.astype(np.int64) * g + c
            span = span * g
    if span < max(4 * key.size, 1 << 20):
        return key.astype(np.int32), int(span)
    return _dense(key)


def _dense(key: np.ndarray) -> tuple[np.ndarray, int]:
    uniq, inv = np.unique(key, return_inverse=True)
    return inv.astype(np.int32).ravel(), int(uniq.size)


def _coerce_ref(ref, categories):
    if ref is None:
        return categories[0]
    if len(categories) and not isinstance(categories[0], type(ref)):
        try:
            return type(categories[0])(ref)
        except (ValueError, TypeError):
            return ref
    return ref


class Expansion:
    """The dummy columns a formula's ``var:i(factor)`` and ``i(var)`` terms expand into
    (polars_impl.py:27-115), planned once from the whole factor columns and applied to any row
    range, so that a streamed (out-of-core) fit expands each chunk as it arrives, as the
    reference expands its scanned LazyFrame lazily (polars_impl.py:342-365).

    ``terms``: (name, var or None, factor, category) in the reference's column order (the
    interactions' columns, then the factors'); ``var`` None is a plain dummy."""

    def __init__(self, factors: dict[str, np.ndarray], interactions, factor_vars, unique=np.unique):
        self.terms = []
        for var, factor, ref in interactions:
            for cat in _categories(unique(factors[factor]), ref, factor):
                self.terms.append((f"{var}_{cat}", var, factor, cat))
        for var, ref in factor_vars:
            for cat in _categories(unique(factors[var]), ref, var):
                self.terms.append((f"{var}_{cat}", None, var, cat))

    @property
    def names(self) -> list[str]:
        return [t[0] for t in self.terms]

    @property
    def numeric_sources(self) -> list[str]:
        """The numeric columns the interaction terms multiply (streamed with the chunks)."""
        return list(dict.fromkeys(t[1] for t in self.terms if t[1] is not None))

    def columns(self, factors: dict[str, np.ndarray], values: dict[str, np.ndarray], rows: slice | None = None,
                which: list[int] | None = None):
        """The expanded columns for one row range: ``factors`` hold the whole factor columns
        (sliced by ``rows``), ``values`` the interactions' numeric columns of that range;
        ``which``: only these terms (indices into ``terms``)."""
        sl = rows if rows is not None else slice(None)
        out = []
        for _, var, factor, cat in (self.terms if which is None else [self.terms[i] for i in which]):
            hit = np.asarray(factors[factor])[sl] == cat
            out.append(np.asarray(values[var], dtype=np.float64) * hit if var is not None else hit.astype(np.float64))
        return out


def _categories(cats, ref, name):
    ref_cat = _coerce_ref(ref, cats)
    if ref_cat not in cats:
        raise ValueError(f"Reference category '{ref}' not found in {name}. Available: {list(cats)}")
    return [cat for cat in cats if cat != ref_cat]


def expand_interactions(cols: dict[str, np.ndarray], interactions, unique=np.unique) -> list[str]:
    """``var:i(factor)`` -> var * (factor == cat) for cat != ref (polars_impl.py:72-115)."""
    plan = Expansion(cols, interactions, [], unique)
    for name, col in zip(plan.names, plan.columns(cols, cols)):
        cols[name] = col
    return plan.names


def expand_factors(cols: dict[str, np.ndarray], factor_vars, unique=np.unique) -> list[str]:
    """``i(var)`` -> dummies (var == cat) for cat != ref (polars_impl.py:27-69)."""
    plan = Expansion(cols, [], factor_vars, unique)
    for name, col in zip(plan.names, plan.columns(cols, cols)):
        cols[name] = col
    return plan.names
