"""The engine reads no environment variables: kernel-path switches are test / A-B knobs set only
through lfe_test_set_knob (a stray variable must not change which kernels run, or the
bit-reproducibility of DESIGN.md §5 would depend on the user's environment).

GPU: every knob name the sources hold is put into the process environment with a value that
would move the path if it were read, and BASELINE configs 1 and 3 (full size, bench.solve_step:
the exact step bench.py times) must give the very bits of the clean environment.  Then the same
names set as knobs do move the path (so the check above is not vacuous)."""
from __future__ import annotations

import glob
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# a value per knob that differs from the production choice wherever the knob is read
ENV_VALUES = {
    "LFE_DENSE": "0", "LFE_DN8": "0", "LFE_DN_PRE": "0", "LFE_DN_C8": "1", "LFE_DN_C4": "0",
    "LFE_DN_ROUNDS": "3", "LFE_K2_NP": "1", "LFE_DN8_K1_MIN": "64", "LFE_DN8_TILED": "1",
    "LFE_DN8_TIMING": "1", "LFE_SWEEP_TIMING": "1", "LFE_K1_UNIT": "256", "LFE_K2_MINROWS": "256",
    "LFE_PART_CW": "4096", "LFE_SUMS_CG": "0", "LFE_TAB3": "0", "LFE_GRAM_GEN": "0", "LFE_GRAM_GU": "2",
    "LFE_CHOL_SPLIT": "1", "LFE_SEG_SORTED": "0", "LFE_SEG_SCATTER_ROWS": "1", "LFE_D3_BATCH": "0",
    "LFE_CL_FIX": "0", "LFE_CL_FUSED": "0", "LFE_CL_STATS": "1", "LFE_CL_NO_SINGLETON": "1",
    "LFE_CL_OWNER_MIN_SPAN": "0", "LFE_CL_MULTI_GATHER": "1", "LFE_ROW_HASH_BITS": "8", "LFE_STR_HASH_BITS": "8", "LFE_HOST_MSG": "1", "LFE_BSTART_MAIN_ROWS": "0", "LFE_H2D_SDMA": "1",
}


def _knob_names() -> set:
    names = set()
    for p in glob.glob(os.path.join(ROOT, "leanfe_amd", "csrc", "*.hip")):
        names |= set(re.findall(r'knob\("([A-Z0-9_]+)"', open(p).read()))
    return names


def test_engine_sources_read_no_environment():
    """No getenv in the engine; every knob the sources read has a test value above."""
    for p in glob.glob(os.path.join(ROOT, "leanfe_amd", "csrc", "*")):
        if os.path.isfile(p):
            assert "getenv" not in open(p, errors="replace").read(), p
    names = _knob_names()
    assert names and names <= set(ENV_VALUES), names - set(ENV_VALUES)


def _solve(cfg):
    import bench
    from leanfe_amd import synth
    from leanfe_amd._lib import Engine

    c = bench.CONFIGS[cfg]
    with Engine(0) as eng:
        eng.synth_load(c["rows"], c["k"], c["levels"], synth.betas(c["k"]), seed=12345)
        r = bench.solve_step(eng, c["vcov"])
        cells = eng.dense_cells()
    return r, cells


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("cfg", [1, 3])
def test_environment_variables_do_not_change_the_bits(cfg, monkeypatch, knob):
    base, cells = _solve(cfg)
    for name in _knob_names():
        monkeypatch.setenv(name, ENV_VALUES[name])
    env, env_cells = _solve(cfg)
    assert env["iterations"] == base["iterations"] and env["n_obs"] == base["n_obs"]
    assert env_cells == cells
    np.testing.assert_array_equal(env["beta"], base["beta"])
    np.testing.assert_array_equal(env["se"], base["se"])
    # the same switch as a knob does move the path: the row sweeps instead of the count tables
    # (config 3) / the count tables forced (config 1), with results at the rounding level only
    knob.setenv("LFE_DENSE", "0" if cells else "1")
    moved, moved_cells = _solve(cfg)
    assert (moved_cells == 0) == bool(cells)
    assert moved["iterations"] == base["iterations"]
    np.testing.assert_allclose(moved["beta"], base["beta"], rtol=1e-10, atol=0)


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("cfg", [1, 3])
def test_host_messages_give_the_same_bits(cfg, knob):
    """LFE_HOST_MSG=1 (off by default: measured slower, profiles/r06/ab_hostmsg.txt): the drop counts,
    bucket starts, stop tests and the residual pass's result block reach the host through mapped host
    words the kernels store, instead of copies - the same values, so the same bits."""
    base, cells = _solve(cfg)
    knob.setenv("LFE_HOST_MSG", "1")
    msg, msg_cells = _solve(cfg)
    assert (msg["iterations"], msg["n_obs"], msg_cells) == (base["iterations"], base["n_obs"], cells)
    np.testing.assert_array_equal(msg["beta"], base["beta"])
    np.testing.assert_array_equal(msg["se"], base["se"])
