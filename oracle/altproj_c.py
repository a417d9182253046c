"""ctypes wrapper of oracle/altproj_c.c — TEST / BASELINE INFRASTRUCTURE ONLY.

``build()`` compiles the C restatement with gcc + OpenMP into oracle/_build/;
``fit_c()`` runs it on host columns (unweighted, IID or HC1).  Only tests/,
__graft_entry__ and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

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


def _load():
    global _lib
    if _lib is None:
        lib = C.CDLL(build())
        lib.lfe_oracle_fit.restype = C.c_int
        lib.lfe_oracle_fit.argtypes = [C.c_int64, C.c_int, C.POINTER(C.c_void_p), C.c_int, C.POINTER(C.c_void_p),
                                       C.POINTER(C.c_int32), C.c_double, C.c_int, C.c_int, C.c_int,
                                       C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int32),
                                       C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        _lib = lib
    return _lib


def fit_c(cols: list[np.ndarray], codes: list[np.ndarray], levels: list[int], *, vcov: str = "iid",
          tol: float = 1e-6, max_iter: int = 50, threads: int = 0) -> dict:
    """cols = [y, x1..xk] (f64), codes = FE codes (int32, dense 0..G-1)."""
    lib = _load()
    cols = [np.ascontiguousarray(c, dtype=np.float64) for c in cols]
    codes = [np.ascontiguousarray(c, dtype=np.int32) for c in codes]
    n, p, F = len(cols[0]), len(cols), len(codes)
    k = p - 1
    cp = (C.c_void_p * p)(*[c.ctypes.data for c in cols])
    kp = (C.c_void_p * F)(*[c.ctypes.data for c in codes])
    lv = (C.c_int32 * F)(*[int(g) for g in levels])
    beta, se = np.zeros(k), np.zeros(k)
    it, nobs, df = C.c_int32(), C.c_int64(), C.c_int64()
    rc = lib.lfe_oracle_fit(n, p, cp, F, kp, lv, float(tol), int(max_iter), 1 if vcov.lower() == "hc1" else 0,
                            int(threads), beta.ctypes.data_as(C.POINTER(C.c_double)),
                            se.ctypes.data_as(C.POINTER(C.c_double)), C.byref(it), C.byref(nobs), C.byref(df))
    if rc != 0:
        raise RuntimeError(f"lfe_oracle_fit failed ({rc})")
    return dict(beta=beta, se=se, iterations=int(it.value), n_obs=int(nobs.value), df_resid=int(df.value))
