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


def test_fa_surf_phase_degenerate():
    """The surf step's degenerate scenes (_scenes.fa_degenerate_surf_pairs): a degenerate iteration
    0 leaves the pose and stops the step; a step with fewer than 10 correspondences skips every
    iteration and passes the carried-in flag through (the corner step skips too)."""
    cfg, cases = _scenes.fa_degenerate_surf_pairs()
    n_deg = n_skip = 0
    for sharp, flat, cl, sl, t0, deg_in in cases:
        o = oracle_py.scan2scan(cfg, sharp, flat, cl, sl, t0, deg_in)
        assert o["corner_iterations"] == 100 and o["n_corner_corr"] < 10
        np.testing.assert_array_equal(o["transform_cur"], t0)  # nothing moves in either case
        if o["n_surf_corr"] >= 10:
            assert o["degenerate"] == 1 and o["surf_iterations"] == 0
            n_deg += 1
        else:
            assert o["surf_iterations"] == 100 and o["degenerate"] == deg_in
            n_skip += 1
    assert n_deg == 2 * len(_scenes.FA_DEGENERATE_SURF_CASES)
    assert n_skip == 2 * len(_scenes.FA_SURF_SKIP_CASES)


def test_moving_drive_iterates_surf_step():
    """synth.sensor_attitude makes consecutive frames differ in z / roll / pitch, so the surf step
    runs past its first iteration (on a level drive it converges at iteration 0)."""
    from llsr import synth
    cfg = default_config("vlp16")
    its = {}
    for motion in (False, True):
        ora = oracle_py.Oracle(cfg)
        prev = ora.process(synth.make_scan(2, "vlp16", motion=motion))
        cur = ora.process(synth.make_scan(3, "vlp16", motion=motion))
        its[motion] = oracle_py.scan2scan(cfg, *oracle_py.fa_lm_inputs(prev, cur), np.zeros(6, np.float32))
    assert its[False]["surf_iterations"] <= 1
    assert its[True]["surf_iterations"] >= 6
