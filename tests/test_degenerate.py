"""CPU: the degenerate branch of both LMs as the oracle restates it (FA:1959-1990, MO:1507-1537).

The eigenvalues are scanned from the largest down (the loop breaks at the first one above the
threshold), so the branch fires only when all of them are below it; every row of matV2 is then
zeroed, matP = matV.inverse() * matV2 and matX = matP * matX2 are zeros, the pose stays put and the
LM stops at iteration 0. The scenes of tests/_scenes.py reach it; the GPU tests compare the device
on the same scenes bit for bit (test_gpu_fa_lm.py, test_gpu_mo.py, test_gpu_shard.py)."""
import numpy as np

import _scenes
import oracle_py
from llsr import _abi, default_config


def test_fa_corner_phase_degenerate():
    cfg, pairs = _scenes.fa_degenerate_pairs()
    n_deg = 0
    for sharp, flat, cl, sl, t0 in pairs:
        o = oracle_py.scan2scan(cfg, sharp, flat, cl, sl, t0, 0)
        if o["degenerate"]:
            n_deg += 1
            assert o["corner_iterations"] == 0  # matX == 0 -> converged at iteration 0
            # the corner phase (ry, tx, tz) did not move transformCur
            surf_only = oracle_py.scan2scan(cfg, sharp[:0], flat, cl, sl, t0, 0)
            assert surf_only["corner_iterations"] == 100 and surf_only["n_corner_corr"] == 0
            np.testing.assert_array_equal(o["transform_cur"][[1, 3, 5]], surf_only["transform_cur"][[1, 3, 5]])
    assert n_deg >= 4


def test_mo_degenerate_freezes_pose():
    cfg = default_config("vlp16")
    for mode in (_abi.LLSR_MODE_LM_APPLIED, _abi.LLSR_MODE_FAITHFUL):
        cfg.mode = mode
        for pr in _scenes.mo_degenerate_problems():
            o = oracle_py.scan2map(cfg, *pr)
            assert o["degenerate"] == 1 and o["iterations"] == 1 and o["converged"] == 1
            assert o["n_corner_corr"] + o["n_surf_corr"] >= 50 and o["min_lambda"] < 100
            np.testing.assert_array_equal(o["pose"], pr[4])
        for pr in _scenes.mo_degenerate_problems(regular=True)[len(_scenes.MO_DEGENERATE_CASES):]:
            assert oracle_py.scan2map(cfg, *pr)["degenerate"] == 0
