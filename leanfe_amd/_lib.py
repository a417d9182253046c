"""ctypes binding of ``liblfe_hip.so`` (C ABI declared in ``include/leanfe_hip.h``).

ctypes releases the GIL for every foreign call.  The engine is the only
compute path of the ``hip`` backend: if the shared library is missing or no
GPU is visible, every entry point raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LEANFE_HIP_LIB") or os.path.join(_HERE, "liblfe_hip.so")

LFE_OK, LFE_EINVAL, LFE_EHIP, LFE_ERCCL, LFE_ENOMEM, LFE_ESTATE, LFE_ENEEDPASS = 0, -1, -2, -3, -4, -5, -6


class NeedsStreamPass(RuntimeError):
    """Streamed X: the Gram from the group tables is unavailable; stream pass 3."""
LFE_HOST, LFE_DEVICE = 0, 1

_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_dp = C.POINTER(C.c_double)
_vp = C.c_void_p

# name -> (restype, argtypes); must match include/leanfe_hip.h
SIGNATURES = {
    "lfe_ctx_create": (C.c_int, [C.POINTER(_vp), C.c_int]),
    "lfe_ctx_destroy": (None, [_vp]),
    "lfe_comm_unique_id": (C.c_int, [_vp]),
    "lfe_ctx_set_comm": (C.c_int, [_vp, _vp, C.c_int, C.c_int]),
    "lfe_emu_create": (C.c_int, [C.c_int, C.POINTER(_vp)]),
    "lfe_emu_destroy": (None, [_vp]),
    "lfe_emu_abort": (None, [_vp]),
    "lfe_ctx_set_emu": (C.c_int, [_vp, _vp, C.c_int]),
    "lfe_load": (C.c_int, [_vp, C.c_int64, C.c_int, C.POINTER(_vp), C.c_int, C.POINTER(_vp), _i32p, _vp, C.c_int]),
    "lfe_load_begin": (C.c_int, [_vp, C.c_int64, C.c_int, C.c_int, _i32p, C.c_int]),
    "lfe_load_rows": (C.c_int, [_vp, C.c_int64, C.c_int64, C.POINTER(_vp), C.POINTER(_vp), _vp]),
    "lfe_load_finish": (C.c_int, [_vp]),
    "lfe_synth_load": (C.c_int, [_vp, C.c_int64, C.c_int, C.c_int, _i32p, _dp, C.c_uint64, C.c_int64]),
    "lfe_ctx_set_owner": (C.c_int, [_vp, C.c_int, C.c_int32, C.c_int32]),
    "lfe_reshard_owner": (C.c_int, [_vp, C.c_int, _i32p, _i32p]),
    "lfe_synth_load_owned": (C.c_int, [_vp, C.c_int64, C.c_int, C.c_int, _i32p, _dp, C.c_uint64, C.c_int,
                                       C.c_int32, C.c_int32]),
    "lfe_load_clusters": (C.c_int, [_vp, C.c_int, C.POINTER(_vp), _i32p, C.c_int]),
    "lfe_drop_singletons": (C.c_int, [_vp, _i64p, _i32p, _i32p]),
    "lfe_demean": (C.c_int, [_vp, _i32p, C.c_double, C.c_int, C.c_int, _i32p, _dp]),
    "lfe_gram": (C.c_int, [_vp, _dp]),
    "lfe_resid": (C.c_int, [_vp, _dp, _dp, _dp, C.c_int]),
    "lfe_resid_iv": (C.c_int, [_vp, _dp, _dp, _dp, C.c_int]),
    "lfe_gram_resid": (C.c_int, [_vp, _dp, _dp, _dp, _dp, C.c_int]),
    "lfe_fit": (C.c_int, [_vp, C.c_int, C.c_double, C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                          _vp]),
    "lfe_cluster_meat": (C.c_int, [_vp, _dp, _i64p]),
    "lfe_cluster_meat_subsets": (C.c_int, [_vp, C.c_int, _vp, _dp, _i64p]),
    "lfe_factorize_ids": (C.c_int, [_vp, C.c_int64, _vp, _vp, C.POINTER(C.c_int32)]),
    "lfe_factorize_strings": (C.c_int, [_vp, C.c_int64, _vp, _vp, _vp, C.POINTER(C.c_int32)]),
    "lfe_count_distinct_rows": (C.c_int, [_vp, C.c_int, _i64p]),
    "lfe_compress": (C.c_int, [_vp, _i64p]),
    "lfe_copy_demeaned": (C.c_int, [_vp, C.POINTER(_vp), _i64p]),
    "lfe_copy_inputs": (C.c_int, [_vp, C.POINTER(_vp), C.POINTER(_vp)]),
    "lfe_exact_sums": (C.c_int, [_vp, _i32p]),
    "lfe_dense_cells": (C.c_int, [_vp, _i64p]),
    "lfe_ctx_test_hooks": (C.c_int, [_vp, C.c_int]),
    "lfe_test_set_knob": (C.c_int, [C.c_char_p, C.c_char_p]),
    "lfe_int_range": (C.c_int, [C.c_void_p, C.c_int64, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "lfe_dev_alloc": (C.c_int, [_vp, C.c_int64, C.POINTER(_vp)]),
    "lfe_dev_free": (C.c_int, [_vp, _vp]),
    "lfe_materialize": (C.c_int, [_vp, _vp, C.c_int64, C.c_int, C.c_int, C.c_int]),
    "lfe_stream_materialize": (C.c_int, [_vp, _vp, C.c_int64, C.c_int, C.c_int]),
    "lfe_stream_materialize_rows": (C.c_int, [_vp, _vp, C.c_int64, C.c_int, C.c_int, C.c_int64, C.c_int64]),
    "lfe_wide_gram_rows": (C.c_int, [_vp, _vp, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, _vp, _dp]),
    "lfe_wide_resid_rows": (C.c_int, [_vp, _vp, C.c_int64, C.c_int64, C.c_int64, C.c_int, _dp, _vp, _dp]),
    "lfe_stream_synth_cols": (C.c_int, [_vp, C.c_int64, C.c_int64, C.c_int, C.c_int, _i32p, _dp, C.c_uint64]),
    "lfe_wide_gram": (C.c_int, [_vp, _vp, C.c_int64, C.c_int, C.c_int, C.c_int, _vp, _dp]),
    "lfe_wide_resid": (C.c_int, [_vp, _vp, C.c_int64, C.c_int, _dp, _vp, _dp]),
    "lfe_wide_cluster_meats": (C.c_int, [_vp, _vp, C.c_int64, C.c_int, C.c_int, _vp, C.c_int, _i32p, _dp, _i64p]),
    "lfe_synth_load_codes_at": (C.c_int, [_vp, C.c_int64, C.c_int64, C.c_int, C.c_int, _i32p, C.c_uint64]),
    "lfe_dense_cell_bytes": (C.c_int, [_vp, C.POINTER(C.c_int32)]),
    "lfe_load_codes": (C.c_int, [_vp, C.c_int64, C.c_int, C.c_int, C.POINTER(_vp), _i32p, _dp, C.c_int]),
    "lfe_stream_clusters": (C.c_int, [_vp, C.c_int, _i32p]),
    "lfe_stream_cluster_meats": (C.c_int, [_vp, _dp, _i64p]),
    "lfe_stream_begin": (C.c_int, [_vp, C.c_int, _dp]),
    "lfe_stream_rows": (C.c_int, [_vp, C.c_int64, C.c_int64, C.POINTER(_vp), C.c_int]),
    "lfe_stream_end": (C.c_int, [_vp, _dp]),
    "lfe_synth_load_codes": (C.c_int, [_vp, C.c_int64, C.c_int, C.c_int, _i32p, C.c_uint64]),
    "lfe_stream_synth_rows": (C.c_int, [_vp, C.c_int64, C.c_int64, C.c_int, _i32p, _dp, C.c_uint64]),
    "lfe_sync": (C.c_int, [_vp]),
    "lfe_shard_rows": (C.c_int, [_vp, _i64p]),
    "lfe_timings": (C.c_int, [_vp, _dp]),
    "lfe_phase_timing": (C.c_int, [_vp, C.c_int]),
    "lfe_profile": (C.c_int, [_vp, C.c_int]),
    "lfe_kernel_stats": (C.c_int, [_vp, C.c_int, C.c_char_p, _dp, _i64p, _i32p]),
    "lfe_last_error": (C.c_char_p, []),
    "lfe_version": (C.c_char_p, []),
    "lfe_build_hash": (C.c_char_p, []),
}

_lock = threading.Lock()
_lib = None


def load_library(path: str | None = None) -> C.CDLL:
    """Load (once) and type the engine library; raises ImportError if absent."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise ImportError(
                f"leanfe_amd HIP engine not found at {p}; build it with `python -m leanfe_amd.build`")
        if path is None and os.environ.get("LFE_ALLOW_STALE") != "1":
            # the library must be built from the sources checked out beside it (build.py stamps
            # their hash into it): a stale build never runs silently
            from .build import library_hash, source_hash
            have, want = library_hash(p), source_hash()
            if have != want:
                raise ImportError(f"{p} was built from other sources (library {have}, sources {want}); "
                                  "rebuild it with `python -m leanfe_amd.build`")
        lib = C.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib


def int_range(values: np.ndarray) -> tuple[int, int]:
    """(min, max) of a signed integer array in one multi-threaded pass (lfe_int_range, host only)."""
    v = np.ascontiguousarray(values)
    lo, hi = C.c_int64(), C.c_int64()
    _check(load_library().lfe_int_range(v.ctypes.data_as(C.c_void_p), v.size, v.dtype.itemsize, C.byref(lo),
                                        C.byref(hi)))
    return int(lo.value), int(hi.value)


def set_knob(name: str, value: str | None) -> None:
    """Set (or with None remove) an engine test / A-B knob (lfe_test_set_knob).  The engine reads no
    environment variables; tests and ``bench.py --knob NAME=VALUE`` use this instead."""
    lib = load_library()
    _check(lib.lfe_test_set_knob(name.encode(), None if value is None else str(value).encode()))


def clear_knobs() -> None:
    _check(load_library().lfe_test_set_knob(b"*", None))


def _check(rc: int) -> None:
    if rc == LFE_OK:
        return
    msg = (load_library().lfe_last_error() or b"").decode(errors="replace")
    if rc == LFE_EINVAL:
        raise ValueError(msg)
    if rc == LFE_ENOMEM:
        raise MemoryError(msg)
    if rc == LFE_ENEEDPASS:
        raise NeedsStreamPass(msg)
    raise RuntimeError(f"leanfe HIP engine error {rc}: {msg}")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class Engine:
    """One engine context on one GPU (one HIP stream, optional RCCL comm)."""

    def __init__(self, device: int = 0):
        self._lib = load_library()
        h = _vp()
        _check(self._lib.lfe_ctx_create(C.byref(h), int(device)))
        self._h = h
        self.device = device
        self.p = 0
        self.F = 0
        self.n = 0  # rows of the loaded shard
        self.owner = None  # (fe, lo, hi) of owner-sharded rows (set_owner / reshard_owner)
        self._keep = []  # host arrays that must outlive async copies

    # -- lifecycle ---------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.lfe_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- distributed -------------------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_char * 128)()
        _check(load_library().lfe_comm_unique_id(C.cast(buf, _vp)))
        return bytes(buf)

    def set_comm(self, unique_id: bytes | None, rank: int, world: int) -> None:
        if world > 1:
            buf = (C.c_char * 128).from_buffer_copy(unique_id)
            _check(self._lib.lfe_ctx_set_comm(self._h, C.cast(buf, _vp), rank, world))
        else:
            _check(self._lib.lfe_ctx_set_comm(self._h, None, 0, 1))

    def set_emu(self, group: "EmuGroup", rank: int) -> None:
        """Join an in-process emulated group (tests of the multi-rank paths on one GPU)."""
        _check(self._lib.lfe_ctx_set_emu(self._h, group.handle, int(rank)))
        self._emu = group  # keep the group alive while this context uses it

    # -- data --------------------------------------------------------------
    def load(self, cols: list[np.ndarray], codes: list[np.ndarray], levels: list[int],
             weights: np.ndarray | None = None) -> None:
        cols = [np.ascontiguousarray(c, dtype=np.float64) for c in cols]
        codes = [np.ascontiguousarray(c, dtype=np.int32) for c in codes]
        n = cols[0].size if cols else 0
        for a in cols + codes:
            if a.size != n:
                raise ValueError("all columns must have the same length")
        w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
        cp = (_vp * len(cols))(*[_ptr(c) for c in cols])
        kp = (_vp * max(len(codes), 1))(*[_ptr(c) for c in codes])
        lv = (C.c_int32 * max(len(levels), 1))(*[int(g) for g in levels])
        _check(self._lib.lfe_load(self._h, n, len(cols), cp, len(codes), kp, lv,
                                  None if w is None else _ptr(w), LFE_HOST))
        self.p, self.F, self.n = len(cols), len(codes), n
        self.owner = None

    # -- chunked upload (streaming ingest) --------------------------------
    def load_begin(self, n: int, p: int, levels: list[int], weighted: bool = False) -> None:
        lv = (C.c_int32 * max(len(levels), 1))(*[int(g) for g in levels])
        _check(self._lib.lfe_load_begin(self._h, int(n), int(p), len(levels), lv, 1 if weighted else 0))
        self.p, self.F, self.n = int(p), len(levels), int(n)
        self.owner = None
        self._inflight = []

    def load_rows(self, row0: int, cols: list[np.ndarray], codes: list[np.ndarray],
                  weights: np.ndarray | None = None) -> None:
        """Rows [row0, row0 + len) of every column; asynchronous (the engine returns once the
        copies of two calls ago are done, so the arrays of the last two calls are kept here)."""
        cols = [np.ascontiguousarray(c, dtype=np.float64) for c in cols]
        codes = [np.ascontiguousarray(c, dtype=np.int32) for c in codes]
        rows = cols[0].size if cols else 0
        if len(cols) != self.p or len(codes) != self.F or any(a.size != rows for a in cols + codes):
            raise ValueError("load_rows: p columns and F code arrays of equal length expected")
        w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
        cp = (_vp * len(cols))(*[_ptr(c) for c in cols])
        kp = (_vp * max(len(codes), 1))(*[_ptr(c) for c in codes])
        _check(self._lib.lfe_load_rows(self._h, int(row0), rows, cp, kp, None if w is None else _ptr(w)))
        self._inflight = (self._inflight + [(cols, codes, w)])[-2:]

    def load_finish(self) -> None:
        _check(self._lib.lfe_load_finish(self._h))
        self._inflight = []

    def synth_load(self, n: int, k: int, levels: list[int], beta: np.ndarray, seed: int = 12345,
                   row_offset: int = 0) -> None:
        lv = (C.c_int32 * max(len(levels), 1))(*[int(g) for g in levels])
        b = np.ascontiguousarray(beta, dtype=np.float64)
        if b.size < max(k, 1):
            b = np.concatenate([b, np.zeros(max(k, 1) - b.size)])
        _check(self._lib.lfe_synth_load(self._h, int(n), int(k), len(levels), lv,
                                        b.ctypes.data_as(_dp), C.c_uint64(seed), int(row_offset)))
        self.p, self.F, self.n = k + 1, len(levels), int(n)
        self.owner = None

    def synth_load_owned(self, n_total: int, k: int, levels: list[int], beta: np.ndarray, owner_fe: int, lo: int,
                         hi: int, seed: int = 12345) -> None:
        """The rows of the synthetic panel [0, n_total) whose code of FE ``owner_fe`` lies in
        [lo, hi), in row order, and owner sharding declared for them (lfe_synth_load_owned)."""
        lv = (C.c_int32 * max(len(levels), 1))(*[int(g) for g in levels])
        b = np.ascontiguousarray(beta, dtype=np.float64)
        if b.size < max(k, 1):
            b = np.concatenate([b, np.zeros(max(k, 1) - b.size)])
        _check(self._lib.lfe_synth_load_owned(self._h, int(n_total), int(k), len(levels), lv,
                                              b.ctypes.data_as(_dp), C.c_uint64(seed), int(owner_fe), int(lo),
                                              int(hi)))
        self.p, self.F = k + 1, len(levels)
        # shard size: copy_inputs needs it; read it back through a zero-cost query
        self.n = self._shard_rows()
        self.owner = (int(owner_fe), int(lo), int(hi))

    def set_owner(self, fe: int | None, lo: int = 0, hi: int = 0) -> None:
        """Declare that this rank holds every row whose code of FE ``fe`` lies in [lo, hi)
        (lfe_ctx_set_owner; None clears it)."""
        _check(self._lib.lfe_ctx_set_owner(self._h, -1 if fe is None else int(fe), int(lo), int(hi)))
        self.owner = None if fe is None else (int(fe), int(lo), int(hi))

    def reshard_owner(self, fe: int) -> tuple[int, int]:
        """Collective: move the loaded rows between the ranks so that this rank holds every row
        whose code of FE ``fe`` lies in the returned level range (balanced by rows), and declare
        owner sharding for it (lfe_reshard_owner)."""
        lo, hi = C.c_int32(), C.c_int32()
        _check(self._lib.lfe_reshard_owner(self._h, int(fe), C.byref(lo), C.byref(hi)))
        self.n = self._shard_rows()
        self.owner = (int(fe), int(lo.value), int(hi.value))
        return int(lo.value), int(hi.value)

    def _shard_rows(self) -> int:
        n = C.c_int64()
        _check(self._lib.lfe_shard_rows(self._h, C.byref(n)))
        return int(n.value)

    def load_clusters(self, codes: list[np.ndarray], levels: list[int]) -> None:
        codes = [np.ascontiguousarray(c, dtype=np.int32) for c in codes]
        kp = (_vp * max(len(codes), 1))(*[_ptr(c) for c in codes])
        lv = (C.c_int32 * max(len(levels), 1))(*[int(g) for g in levels])
        _check(self._lib.lfe_load_clusters(self._h, len(codes), kp, lv, LFE_HOST))
        self._ncl = len(codes)

    # -- host prep on the device --------------------
    def factorize_ids(self, ids: np.ndarray) -> tuple[np.ndarray, int]:
        """Dense int32 codes of an integer id column, sorted-unique order (np.unique's inverse)."""
        a = np.ascontiguousarray(ids, dtype=np.int64)
        codes = np.empty(a.size, dtype=np.int32)
        g = C.c_int32()
        _check(self._lib.lfe_factorize_ids(self._h, a.size, _ptr(a) if a.size else None,
                                           _ptr(codes) if a.size else None, C.byref(g)))
        return codes, int(g.value)

    def factorize_strings(self, offsets: np.ndarray, data: np.ndarray) -> tuple[np.ndarray, int]:
        """Dense int32 codes of a string column in Arrow layout (int64 offsets [n + 1] from 0,
        uint8 bytes): exact grouping, codes numbered in string-hash order."""
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        buf = np.ascontiguousarray(data, dtype=np.uint8)
        n = max(off.size - 1, 0)
        codes = np.empty(n, dtype=np.int32)
        g = C.c_int32()
        _check(self._lib.lfe_factorize_strings(self._h, n, _ptr(off) if n else None,
                                               _ptr(buf) if buf.size else None,
                                               _ptr(codes) if n else None, C.byref(g)))
        return codes, int(g.value)

    def count_distinct_rows(self, n_x: int = -1) -> int:
        """Distinct (x, FE) rows of the loaded data (estimate_compression_ratio's numerator);
        ``n_x`` regressor columns follow y (instruments after them are not part of the key)."""
        out = C.c_int64()
        _check(self._lib.lfe_count_distinct_rows(self._h, int(n_x), C.byref(out)))
        return int(out.value)

    # -- hot path ----------------------------------------------------------
    def drop_singletons(self) -> tuple[int, tuple, tuple]:
        n = C.c_int64()
        dims = (C.c_int32 * max(self.F, 1))()
        card = (C.c_int32 * max(self.F, 1))()
        _check(self._lib.lfe_drop_singletons(self._h, C.byref(n), dims, card))
        return int(n.value), tuple(int(d) for d in dims[:self.F]), tuple(int(c) for c in card[:self.F])

    def demean(self, order: list[int], tol: float = 1e-6, max_iter: int = 50,
               check_from: int = 3) -> tuple[int, float]:
        o = (C.c_int32 * max(len(order), 1))(*order)
        it = C.c_int32()
        last = C.c_double()
        _check(self._lib.lfe_demean(self._h, o, float(tol), int(max_iter), int(check_from),
                                    C.byref(it), C.byref(last)))
        return int(it.value), float(last.value)

    def gram(self) -> np.ndarray:
        m = self.p + 1
        out = np.zeros((m, m))
        _check(self._lib.lfe_gram(self._h, out.ctypes.data_as(_dp)))
        return out

    def resid(self, beta_full: np.ndarray, hc1: bool = False, keep_scores: bool = False):
        b = np.ascontiguousarray(beta_full, dtype=np.float64)
        stats = np.zeros(4)
        k = self.p - 1
        meat = np.zeros((max(k, 1), max(k, 1))) if hc1 else None
        _check(self._lib.lfe_resid(self._h, b.ctypes.data_as(_dp), stats.ctypes.data_as(_dp),
                                   None if meat is None else meat.ctypes.data_as(_dp),
                                   1 if keep_scores else 0))
        if keep_scores:
            self._score_k = k
        return stats, (meat[:k, :k] if meat is not None else None)

    def compress(self) -> int:
        """YOCO: replace the loaded rows (and cluster columns) by their compressed
        records (lfe_compress); returns the number of records."""
        n = C.c_int64()
        _check(self._lib.lfe_compress(self._h, C.byref(n)))
        self.n = int(n.value)
        return self.n

    def resid_iv(self, coef: np.ndarray, meat: bool = False, keep_scores: bool = False):
        """IV residual pass (lfe_resid_iv): r = y~ - coef . [1, cols 1..p-1]; returns
        (stats, p x p meat over u = [1, cols 1..p-1] or None)."""
        c = np.ascontiguousarray(coef, dtype=np.float64)
        if c.shape != (self.p,):
            raise ValueError(f"coef must have p = {self.p} entries")
        stats = np.zeros(4)
        M = np.zeros((self.p, self.p)) if meat else None
        _check(self._lib.lfe_resid_iv(self._h, c.ctypes.data_as(_dp), stats.ctypes.data_as(_dp),
                                      None if M is None else M.ctypes.data_as(_dp), 1 if keep_scores else 0))
        if keep_scores:
            self._score_k = self.p
        return stats, M

    def gram_resid(self, hc1: bool = False, keep_scores: bool = False):
        """Gram + device solve + residual pass in one call (lfe_gram_resid).  Returns
        (gram, beta_full_device, stats, meat) or None when the fused path does not apply."""
        D = self.p + 1
        G = np.zeros((D, D))
        b = np.zeros(self.p)
        stats = np.zeros(4)
        k = self.p - 1
        meat = np.zeros((max(k, 1), max(k, 1))) if hc1 else None
        rc = self._lib.lfe_gram_resid(self._h, G.ctypes.data_as(_dp), b.ctypes.data_as(_dp),
                                      stats.ctypes.data_as(_dp), None if meat is None else meat.ctypes.data_as(_dp),
                                      int(keep_scores))
        if rc == 1:
            return None
        _check(rc)
        if keep_scores:
            self._score_k = k
        return G, b, stats, (meat[:k, :k] if hc1 else None)

    FIT_VCOV = {"iid": 0, "hc1": 1, "cluster": 2}

    def _fit_bufs(self, v: int, drop: bool, tol: float, max_iter: int, check_from: int):
        """Output buffers and the ctypes argument tuple of lfe_fit, built once per shape and options
        (the call sits between two solves on the GPU's critical path: ~20 us of argument conversion
        and allocation per call otherwise)."""
        if self._h is None:
            raise RuntimeError("engine is closed")
        h = self._h.value if isinstance(self._h, C.c_void_p) else self._h
        key = (h, self.F, self.p, v, drop, tol, max_iter, check_from)
        cache = self.__dict__.setdefault("_fit_cache", {})
        hit = cache.get(key)
        if hit is not None:
            return hit
        F, p = self.F, self.p
        k, D = p - 1, p + 1
        ints = np.zeros(4 + 2 * F, dtype=np.int64)
        buf = np.zeros(D * D + p + p * p + 4 + k * k + k + 2)
        o = [int(x) for x in np.cumsum([0, D * D, p, p * p, 4, k * k, k])]
        b = buf.ctypes.data
        args = (C.c_void_p(h), C.c_int(1 if drop else 0), C.c_double(tol), C.c_int(max_iter),
                C.c_int(check_from), C.c_int(v), C.c_void_p(ints.ctypes.data),
                *[C.c_void_p(b + 8 * o[i]) for i in range(7)])
        fn = self._lib.lfe_fit
        hit = cache[key] = (fn, args, ints, buf, o)
        return hit

    def fit(self, vcov: str, tol: float = 1e-6, max_iter: int = 50, check_from: int = 3, drop: bool = True) -> dict:
        """One whole regression in one C call (lfe_fit): [singleton drop], projections with the FEs
        ordered by cardinality, Gram + device solve + residual pass, host solve and the IID / HC1
        SEs; 'cluster' keeps the score rows for cluster_meat* (se is then None).  Unweighted,
        resident, no instruments.  The returned arrays are copies."""
        v = self.FIT_VCOV[vcov.lower()]
        fn, args, ints, buf, o = self._fit_bufs(v, drop, float(tol), int(max_iter), int(check_from))
        _check(fn(*args))
        F, p = self.F, self.p
        k, D = p - 1, p + 1
        if v == 2:
            self._score_k = k
        out = buf.copy()
        return dict(n_obs=int(ints[0]), iterations=int(ints[1]), df_resid=int(ints[2]), fused=bool(ints[3]),
                    fe_dims=tuple(ints[4:4 + F].tolist()), fe_card=tuple(ints[4 + F:].tolist()),
                    gram=out[:o[1]].reshape(D, D), beta_full=out[o[1]:o[2]], xtx_inv=out[o[2]:o[3]].reshape(p, p),
                    stats=out[o[3]:o[4]], meat=out[o[4]:o[5]].reshape(k, k) if v == 1 else None,
                    se=out[o[5]:o[6]] if v != 2 else None, last_check=float(out[o[6]]),
                    beta_dev_vs_host=float(out[o[6] + 1]))

    def cluster_meat(self) -> tuple[np.ndarray, np.ndarray]:
        k = getattr(self, "_score_k", self.p - 1)
        m = self._ncl
        meats = np.zeros(max(m * k * k, 1))
        G = np.zeros(max(m, 1), dtype=np.int64)
        _check(self._lib.lfe_cluster_meat(self._h, meats.ctypes.data_as(_dp), G.ctypes.data_as(_i64p)))
        return meats[:m * k * k].reshape(m, k, k), G[:m]

    def cluster_meat_subsets(self, subsets) -> tuple[np.ndarray, np.ndarray]:
        """CGM subsets (tuples of loaded cluster column indices) grouped on the device."""
        k = getattr(self, "_score_k", self.p - 1)
        masks = np.array([sum(1 << j for j in s) for s in subsets], dtype=np.int32)
        m = len(masks)
        meats = np.zeros(max(m * k * k, 1))
        G = np.zeros(max(m, 1), dtype=np.int64)
        _check(self._lib.lfe_cluster_meat_subsets(self._h, m, masks.ctypes.data_as(_vp),
                                                  meats.ctypes.data_as(_dp), G.ctypes.data_as(_i64p)))
        return meats[:m * k * k].reshape(m, k, k), G[:m]

    def _rows(self, n: int | None) -> int:
        # the engine always copies every row of the loaded shard
        if n is not None and int(n) != self.n:
            raise ValueError(f"n={n} but the loaded shard has {self.n} rows")
        return self.n

    def copy_demeaned(self, n: int | None = None) -> np.ndarray:
        n = self._rows(n)
        out = np.zeros((self.p, n))
        ptrs = (_vp * self.p)(*[out[j].ctypes.data for j in range(self.p)])
        nn = C.c_int64()
        _check(self._lib.lfe_copy_demeaned(self._h, ptrs, C.byref(nn)))
        return out

    def copy_inputs(self, n: int | None = None) -> tuple[np.ndarray, np.ndarray]:
        n = self._rows(n)
        cols = np.zeros((self.p, n))
        codes = np.zeros((max(self.F, 1), n), dtype=np.int32)
        cp = (_vp * self.p)(*[cols[j].ctypes.data for j in range(self.p)])
        kp = (_vp * max(self.F, 1))(*[codes[f].ctypes.data for f in range(max(self.F, 1))])
        _check(self._lib.lfe_copy_inputs(self._h, cp, kp))
        return cols, codes[:self.F]

    def sync(self) -> None:
        _check(self._lib.lfe_sync(self._h))

    # -- out-of-core X: codes resident, columns streamed in row chunks ----
    def load_codes(self, codes: list[np.ndarray], levels: list[int], p: int,
                   weights: np.ndarray | None = None) -> None:
        """FE codes (and weights) of n rows (input order); the p data columns come later in chunks."""
        codes = [np.ascontiguousarray(c, dtype=np.int32) for c in codes]
        n = codes[0].size if codes else 0
        kp = (_vp * max(len(codes), 1))(*[_ptr(c) for c in codes])
        lv = (C.c_int32 * max(len(levels), 1))(*[int(g) for g in levels])
        w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
        _check(self._lib.lfe_load_codes(self._h, n, int(p), len(codes), kp, lv,
                                        None if w is None else w.ctypes.data_as(_dp), LFE_HOST))
        self.p, self.F, self.n = int(p), len(codes), n
        self.owner = None

    def stream_begin(self, pass_: int, beta_full: np.ndarray | None = None) -> None:
        b = None if beta_full is None else np.ascontiguousarray(beta_full, dtype=np.float64)
        _check(self._lib.lfe_stream_begin(self._h, int(pass_), None if b is None else
                                          b.ctypes.data_as(C.POINTER(C.c_double))))

    def stream_rows(self, row0: int, cols: list[np.ndarray]) -> None:
        cols = [np.ascontiguousarray(c, dtype=np.float64) for c in cols]
        rows = cols[0].size if cols else 0
        if len(cols) != self.p or any(c.size != rows for c in cols):
            raise ValueError(f"stream_rows needs {self.p} columns of equal length")
        cp = (_vp * len(cols))(*[_ptr(c) for c in cols])
        _check(self._lib.lfe_stream_rows(self._h, int(row0), rows, cp, LFE_HOST))

    def stream_clusters(self, subsets: list[int]) -> None:
        """Factorize every cluster subset (bit mask over the loaded cluster columns) for the
        streamed residual passes' score sums (lfe_stream_clusters)."""
        m = (C.c_int32 * len(subsets))(*[int(s) for s in subsets])
        _check(self._lib.lfe_stream_clusters(self._h, len(subsets), m))
        self._stream_subsets = len(subsets)

    def stream_cluster_meats(self, ks: int) -> tuple[np.ndarray, np.ndarray]:
        """(meats [n_subsets][ks][ks], cluster counts) after a streamed residual pass."""
        ns = self._stream_subsets
        meats = np.zeros((ns, ks, ks), dtype=np.float64)
        G = np.zeros(ns, dtype=np.int64)
        _check(self._lib.lfe_stream_cluster_meats(self._h, meats.ctypes.data_as(_dp), G.ctypes.data_as(_i64p)))
        return meats, G

    def stream_end(self) -> np.ndarray:
        out = np.zeros(max(4 + self.p ** 2, (self.p + 1) ** 2), dtype=np.float64)
        _check(self._lib.lfe_stream_end(self._h, out.ctypes.data_as(C.POINTER(C.c_double))))
        return out

    def synth_load_codes(self, n: int, k: int, levels: list[int], seed: int = 12345, row0: int = 0) -> None:
        """Codes of rows [row0, row0 + n) of the synthetic panel (lfe_synth_load_codes_at); the
        columns come later, generated chunk by chunk (stream_synth_pass)."""
        lv = (C.c_int32 * len(levels))(*[int(g) for g in levels])
        _check(self._lib.lfe_synth_load_codes_at(self._h, int(n), int(row0), int(k), len(levels), lv,
                                                 C.c_uint64(seed)))
        self.p, self.F, self.n = int(k) + 1, len(levels), int(n)
        self.owner = None

    def stream_synth_pass(self, pass_: int, k: int, levels: list[int], beta: np.ndarray, chunk_rows: int,
                          seed: int = 12345, beta_full: np.ndarray | None = None) -> np.ndarray:
        """One pass whose chunks are the synthetic panel's rows, generated on the device."""
        lv = (C.c_int32 * len(levels))(*[int(g) for g in levels])
        b = np.ascontiguousarray(beta, dtype=np.float64)
        self.stream_begin(pass_, beta_full)
        for r0 in range(0, self.n, chunk_rows):
            rows = min(chunk_rows, self.n - r0)
            _check(self._lib.lfe_stream_synth_rows(self._h, r0, rows, int(k), lv,
                                                   b.ctypes.data_as(C.POINTER(C.c_double)), C.c_uint64(seed)))
        return self.stream_end()

    def stream_pass(self, pass_: int, chunks, beta_full: np.ndarray | None = None) -> np.ndarray:
        """One pass over ``chunks`` (an iterable of (row0, [p columns])) between begin / end."""
        self.stream_begin(pass_, beta_full)
        for row0, cols in chunks:
            self.stream_rows(row0, cols)
        return self.stream_end()

    def exact_sums(self) -> bool:
        """True when the last group sums took the exact int64 path (order-independent)."""
        on = C.c_int32(0)
        _check(self._lib.lfe_exact_sums(self._h, C.byref(on)))
        return bool(on.value)

    # -- wide fits (p > 63: column blocks of contexts, lfe_wide.hip) ------------
    def dev_alloc(self, n_doubles: int) -> int:
        """A zero-filled device buffer of n_doubles (lfe_dev_alloc); release with dev_free."""
        p = _vp()
        _check(self._lib.lfe_dev_alloc(self._h, int(n_doubles), C.byref(p)))
        return p.value

    def dev_free(self, ptr: int) -> None:
        _check(self._lib.lfe_dev_free(self._h, _vp(ptr)))

    def materialize(self, D: int, ldD: int, first: int, col0: int, mask_col: int = -1) -> None:
        """This context's demeaned columns [first, p) into D's columns col0.. (input row order)."""
        _check(self._lib.lfe_materialize(self._h, _vp(D), int(ldD), int(first), int(col0), int(mask_col)))

    def stream_materialize(self, D: int, ldD: int, col0: int, chunks, mask_col: int = -1) -> None:
        """A streamed context's demeaned columns, chunk by chunk, into D's columns col0.. (pass 5)."""
        _check(self._lib.lfe_stream_materialize(self._h, _vp(D), int(ldD), int(col0), int(mask_col)))
        for row0, cols in chunks:
            self.stream_rows(row0, cols)
        _check(self._lib.lfe_stream_end(self._h, None))

    def stream_materialize_rows(self, D: int, ldD: int, col0: int, row0: int, cols, mask_col: int = -1) -> None:
        """Rows [row0, row0 + len) of a streamed context's demeaned columns into D rows 0.. (one chunk of
        a chunked wide fit); ``cols``: the chunk's columns (host arrays) or ("synth", K, c_lo, levels,
        beta, seed) to generate them on the device."""
        if isinstance(cols, tuple) and cols and cols[0] == "synth":
            _, rows, K, c_lo, levels, beta, seed = cols
        else:
            rows = len(cols[0])
        _check(self._lib.lfe_stream_materialize_rows(self._h, _vp(D), int(ldD), int(col0), int(mask_col), int(row0),
                                                     int(rows)))
        if isinstance(cols, tuple) and cols and cols[0] == "synth":
            self.stream_synth_cols(row0, rows, K, c_lo, levels, beta, seed)
        else:
            self.stream_rows(row0, cols)
        _check(self._lib.lfe_stream_end(self._h, None))

    def stream_synth_cols(self, row0: int, rows: int, K: int, c_lo: int, levels, beta, seed: int) -> None:
        lv = (C.c_int32 * max(len(levels), 1))(*[int(g) for g in levels])
        b = np.ascontiguousarray(beta, dtype=np.float64)
        _check(self._lib.lfe_stream_synth_cols(self._h, int(row0), int(rows), int(K), int(c_lo), lv,
                                               b.ctypes.data_as(_dp), C.c_uint64(seed)))

    def wide_gram_rows(self, D: int, ldD: int, row0: int, rows: int, c0: int, P: int, mode: int = 0,
                       r: int | None = None) -> np.ndarray:
        out = np.zeros((P, P))
        _check(self._lib.lfe_wide_gram_rows(self._h, _vp(D), int(ldD), int(row0), int(rows), int(c0), int(P), int(mode),
                                            None if r is None else _vp(r), out.ctypes.data_as(_dp)))
        return out

    def wide_resid_rows(self, D: int, ldD: int, row0: int, rows: int, coef: np.ndarray, r: int) -> np.ndarray:
        v = np.ascontiguousarray(coef, dtype=np.float64)
        stats = np.zeros(4)
        _check(self._lib.lfe_wide_resid_rows(self._h, _vp(D), int(ldD), int(row0), int(rows), int(v.size),
                                             v.ctypes.data_as(_dp), _vp(r), stats.ctypes.data_as(_dp)))
        return stats

    def wide_gram(self, D: int, ldD: int, c0: int, P: int, mode: int = 0, r: int | None = None) -> np.ndarray:
        out = np.zeros((P, P))
        _check(self._lib.lfe_wide_gram(self._h, _vp(D), int(ldD), int(c0), int(P), int(mode),
                                       None if r is None else _vp(r), out.ctypes.data_as(_dp)))
        return out

    def wide_resid(self, D: int, ldD: int, coef: np.ndarray, r: int) -> np.ndarray:
        v = np.ascontiguousarray(coef, dtype=np.float64)
        stats = np.zeros(4)
        _check(self._lib.lfe_wide_resid(self._h, _vp(D), int(ldD), int(v.size), v.ctypes.data_as(_dp), _vp(r),
                                        stats.ctypes.data_as(_dp)))
        return stats

    def wide_cluster_meats(self, D: int, ldD: int, c0: int, k: int, r: int, subsets) -> tuple[np.ndarray, np.ndarray]:
        masks = np.array([sum(1 << j for j in s) for s in subsets], dtype=np.int32)
        m = len(masks)
        meats = np.zeros(max(m * k * k, 1))
        G = np.zeros(max(m, 1), dtype=np.int64)
        _check(self._lib.lfe_wide_cluster_meats(self._h, _vp(D), int(ldD), int(c0), int(k), _vp(r), m,
                                                masks.ctypes.data_as(_i32p), meats.ctypes.data_as(_dp),
                                                G.ctypes.data_as(_i64p)))
        return meats[:m * k * k].reshape(m, k, k), G[:m]

    def test_hooks(self, flags: int) -> None:
        """Test-only switches (lfe_ctx_test_hooks; 1 = LFE_TEST_SHORT_MEMORY: this rank's owner
        re-shard reports too little device memory; 2 = LFE_TEST_CLUSTER_SORTED: one-column cluster
        subsets take the sorted path; 4 = LFE_TEST_CLUSTER_STATS: the sort-free cluster sums take
        their quanta from a statistics pass; 8 = LFE_TEST_SEG_SCATTER: the row sweeps' segment
        layouts are built by the block scatter instead of the sorted build)."""
        _check(self._lib.lfe_ctx_test_hooks(self._h, int(flags)))

    def dense_cells(self) -> int:
        """Cells of the count tables the last two-FE demean multiplied on the matrix cores (0: the row
        layouts ran; lfe_dense.hip)."""
        v = C.c_int64(0)
        _check(self._lib.lfe_dense_cells(self._h, C.byref(v)))
        return int(v.value)


    def dense_cell_bytes(self) -> int:
        """Bytes per cell the dense passes read (1: the exact i8 tables, 2: u16; 0: row layouts)."""
        v = C.c_int32(0)
        _check(self._lib.lfe_dense_cell_bytes(self._h, C.byref(v)))
        return int(v.value)
    def profile(self, enable: bool = True) -> None:
        _check(self._lib.lfe_profile(self._h, 1 if enable else 0))

    def phase_timing(self, enable: bool = True) -> None:
        """Per-phase device times for timings() (off by default: event records cost host time)."""
        _check(self._lib.lfe_phase_timing(self._h, 1 if enable else 0))

    def kernel_stats(self) -> dict:
        """{kernel name: (total ms, launches)} since the last profile(True)."""
        cap = 64
        names = C.create_string_buffer(32 * cap)
        ms = np.zeros(cap)
        cnt = np.zeros(cap, dtype=np.int64)
        n = C.c_int32()
        _check(self._lib.lfe_kernel_stats(self._h, cap, names, ms.ctypes.data_as(_dp),
                                          cnt.ctypes.data_as(_i64p), C.byref(n)))
        raw = names.raw
        out = {}
        for j in range(n.value):
            nm = raw[32 * j:32 * j + 32].split(b"\0", 1)[0].decode()
            out[nm] = (float(ms[j]), int(cnt[j]))
        return out

    def timings(self) -> dict:
        t = np.zeros(6)
        _check(self._lib.lfe_timings(self._h, t.ctypes.data_as(_dp)))
        return dict(zip(["prep", "demean", "gram", "resid", "cluster", "last"], t.tolist()))


def version() -> str:
    return load_library().lfe_version().decode()


class EmuGroup:
    """In-process group of `world` contexts (lfe_emu_create): each context is driven by its own
    thread and the engine's collectives meet at a host barrier.  Used by the tests' emulated ranks
    and by a fit of more rows than one context holds (< 2^31 per context: several contexts on one
    device, hip_impl._out_of_core_split).  ``exchange`` is the host-side all-gather those threads
    use for the level counts and factor categories they must agree on."""

    def __init__(self, world: int):
        import threading

        self._lib = load_library()
        h = _vp()
        _check(self._lib.lfe_emu_create(int(world), C.byref(h)))
        self.handle = h
        self.world = world
        self._barrier = threading.Barrier(int(world))
        self._slots = [None] * int(world)

    def abort(self) -> None:
        """A member failed: the others' waiting and later collectives fail instead of waiting."""
        self._lib.lfe_emu_abort(self.handle)
        self._barrier.abort()

    def exchange(self, rank: int, obj):
        """Every member's ``obj``, in rank order (all members call it, each from its thread)."""
        self._slots[rank] = obj
        self._barrier.wait()
        out = list(self._slots)
        self._barrier.wait()  # every member has read the slots before they are reused
        return out

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            self._lib.lfe_emu_destroy(h)
            self.handle = None
