"""ctypes wrapper of oracle/altproj_c.c — TEST / BASELINE INFRASTRUCTURE ONLY.

``build()`` compiles the C restatement with gcc + OpenMP into oracle/_build/;
``fit_c()`` runs it on host columns (unweighted; IID, HC1, one-way or CGM
multi-way clustered SEs).  Only tests/, tools/ parity runs, __graft_entry__ and
bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from itertools import combinations

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "altproj_c.c")
LIB = os.path.join(HERE, "_build", "libaltproj.so")


def build(force: bool = False) -> str:
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["gcc", "-O3", "-march=x86-64-v2", "-fopenmp", "-shared", "-fPIC", SRC, "-o", LIB, "-lm"],
                   check=True)
    return LIB


_lib = None
_vp = C.c_void_p
_dp = C.POINTER(C.c_double)
_i64p = C.POINTER(C.c_int64)


def _load():
    global _lib
    if _lib is None:
        lib = C.CDLL(build())
        lib.lfe_oracle_fit.restype = C.c_int
        lib.lfe_oracle_fit.argtypes = [
            C.c_int64, C.c_int, C.POINTER(_vp), C.c_int, C.POINTER(_vp), C.POINTER(C.c_int32),  # n, p, cols, F..
            C.c_int, C.POINTER(_vp), C.POINTER(C.c_int32),                                     # m, cl codes, levels
            C.c_double, C.c_int, C.c_int, C.c_int, C.c_int,                                    # tol .. threads
            _dp, _dp, C.POINTER(C.c_int32), _i64p, _i64p, _i64p, _dp, _dp, _i64p]
        _lib = lib
    return _lib


def cluster_subsets(m: int) -> list[tuple[int, ...]]:
    """CGM subsets by size, itertools.combinations order (std_errors.py:392-425)."""
    return [s for size in range(1, m + 1) for s in combinations(range(m), size)]


def default_threads() -> int:
    """Host threads the baseline may use: the scheduler affinity, capped by OMP_NUM_THREADS
    when it is set (GNU ``nproc`` reports the same number)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def fit_c(cols: list[np.ndarray], codes: list[np.ndarray], levels: list[int], *, vcov: str = "iid",
          tol: float = 1e-6, max_iter: int = 50, threads: int = 0, cl_codes: list[np.ndarray] | None = None,
          cl_levels: list[int] | None = None, ssc: bool = True) -> dict:
    """cols = [y, x1..xk] (f64), codes = FE codes (int32, dense 0..G-1); for vcov='cluster'
    cl_codes are dense int32 cluster codes (cl_levels their level counts)."""
    lib = _load()
    cols = [np.ascontiguousarray(c, dtype=np.float64) for c in cols]
    codes = [np.ascontiguousarray(c, dtype=np.int32) for c in codes]
    v = vcov.lower()
    mode = {"iid": 0, "hc1": 1, "cluster": 2}[v]
    cl = [np.ascontiguousarray(c, dtype=np.int32) for c in (cl_codes or [])]
    if mode == 2 and not cl:
        raise ValueError("cluster_cols required for vcov='cluster'")
    if cl and cl_levels is None:
        cl_levels = [int(c.max()) + 1 if c.size else 1 for c in cl]
    n, p, F, m = len(cols[0]), len(cols), len(codes), len(cl)
    k = p - 1
    nsub = (1 << m) - 1
    cp = (_vp * p)(*[c.ctypes.data for c in cols])
    kp = (_vp * max(F, 1))(*[c.ctypes.data for c in codes])
    lv = (C.c_int32 * max(F, 1))(*[int(g) for g in levels])
    clp = (_vp * max(m, 1))(*[c.ctypes.data for c in cl])
    cll = (C.c_int32 * max(m, 1))(*[int(g) for g in (cl_levels or [])])
    beta, se = np.zeros(max(k, 1)), np.zeros(max(k, 1))
    stats = np.zeros(4)
    meats = np.zeros(max(nsub * k * k, 1))
    gsub = np.zeros(max(nsub, 1), dtype=np.int64)
    ncl = np.zeros(max(m, 1), dtype=np.int64)
    it, nobs, df = C.c_int32(), C.c_int64(), C.c_int64()
    rc = lib.lfe_oracle_fit(n, p, cp, F, kp, lv, m, clp, cll, float(tol), int(max_iter), mode, 1 if ssc else 0,
                            int(threads), beta.ctypes.data_as(_dp), se.ctypes.data_as(_dp), C.byref(it),
                            C.byref(nobs), C.byref(df), ncl.ctypes.data_as(_i64p), stats.ctypes.data_as(_dp),
                            meats.ctypes.data_as(_dp), gsub.ctypes.data_as(_i64p))
    if rc != 0:
        raise RuntimeError(f"lfe_oracle_fit failed ({rc})")
    out = dict(beta=beta[:k], se=se[:k], iterations=int(it.value), n_obs=int(nobs.value), df_resid=int(df.value),
               rss=float(stats[0]), tss=float(stats[1]), r_squared=float(stats[2]))
    if mode == 2:
        out["n_clusters"] = int(ncl[0]) if m == 1 else tuple(int(g) for g in ncl[:m])
        out["subsets"] = cluster_subsets(m)
        out["G_subsets"] = [int(g) for g in gsub[:nsub]]
        out["meats"] = meats[:nsub * k * k].reshape(nsub, k, k)
    return out
