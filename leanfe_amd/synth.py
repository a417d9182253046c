"""Counter-based synthetic HDFE panel, host (NumPy) side.

Every value is a pure function of (seed, stream, counter), so the host, the CPU
baseline and any number of GPU row shards see bit-identical inputs.  The device
generator ``lfe_synth_panel`` in ``csrc/lfe_synth.hip`` evaluates exactly the
same expressions, with floating-point contraction disabled, so a row generated
on the GPU equals the row generated here bit for bit.

Definitions (seed defaults to 12345, the reference's cross-language seed,
``tests/test_cross_language_equivalence.py:25``):

* ``key(i, s) = seed ^ (s << 40) ^ i``; ``u(i, s) = ((splitmix64(key) >> 12) + 0.5) * 2^-52``
* ``z(i, s) = (u(i,16s) + u(i,16s+1) + ... + u(i,16s+11)) - 6``   (Irwin-Hall, left to right)
* ``fe_f[i] = min(floor(u(i, f) * L_f), L_f - 1)``
* FE effects: ``a_f[g] = c_f * z(g, 101 + f)`` with ``c = (1, 0.5, 0.25, ...)``
* ``X_ij = z(i, 200 + j) + 0.5 * a_0[fe_0[i]]``
* ``y_i = sum_j beta_j X_ij + sum_f a_f[fe_f[i]] + z(i, 300)``, ``beta = linspace(1, 0.1, k)``
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_MUL1 = np.uint64(0xBF58476D1CE4E5B9)
_MUL2 = np.uint64(0x94D049BB133111EB)
_TWO_M52 = 2.0 ** -52


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _MUL1
        z = (z ^ (z >> np.uint64(27))) * _MUL2
        return z ^ (z >> np.uint64(31))


def uniform(i: np.ndarray, s: int, seed: int) -> np.ndarray:
    key = np.uint64(seed) ^ (np.uint64(s) << np.uint64(40)) ^ np.asarray(i, dtype=np.uint64)
    v = (splitmix64(key) >> np.uint64(12)).astype(np.float64)
    return (v + 0.5) * _TWO_M52


def normal(i: np.ndarray, s: int, seed: int) -> np.ndarray:
    acc = uniform(i, 16 * s, seed)
    for j in range(1, 12):
        acc = acc + uniform(i, 16 * s + j, seed)
    return acc - 6.0


def betas(k: int) -> np.ndarray:
    return np.linspace(1.0, 0.1, k) if k > 1 else np.ones(k)


def fe_effect_scale(f: int) -> float:
    return 0.5 ** f


def panel(n: int, k: int, levels: list[int], seed: int = 12345, row_offset: int = 0) -> dict:
    """Rows ``row_offset .. row_offset+n-1`` of the synthetic panel as a dict of
    NumPy columns: ``y``, ``x1..xk`` (f64) and ``fe1..feF`` (int32)."""
    i = np.arange(row_offset, row_offset + n, dtype=np.uint64)
    out = {}
    codes = []
    for f, L in enumerate(levels):
        c = np.floor(uniform(i, f, seed) * L)
        c = np.minimum(c, L - 1).astype(np.int32)
        codes.append(c)
    eff = []
    for f, L in enumerate(levels):
        g = np.arange(L, dtype=np.uint64)
        eff.append(fe_effect_scale(f) * normal(g, 101 + f, seed))
    a0 = eff[0][codes[0]] if levels else np.zeros(n)
    b = betas(k)
    y = None
    for j in range(k):
        x = normal(i, 200 + j, seed) + 0.5 * a0
        out[f"x{j + 1}"] = x
        t = b[j] * x
        y = t if y is None else y + t
    if y is None:
        y = np.zeros(n)
    for f in range(len(levels)):
        y = y + eff[f][codes[f]]
    y = y + normal(i, 300, seed)
    out["y"] = y
    for f in range(len(levels)):
        out[f"fe{f + 1}"] = codes[f]
    return out
