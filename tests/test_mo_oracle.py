"""CPU checks of the MapOptimization restatement (oracle/oracle_mo.cpp) and the oracle's own
Eigen 3.3.7 restatement (oracle/oracle_eigen.h; the device's is cross-checked against it bit for
bit by tests/test_eigen_restatement.py).

Parity status: the reference's scan-to-map cannot run here (ROS2/PCL/GTSAM absent, SURVEY.md
§8c) and ships no golden vectors for it, so the optimiser itself is "parity unpinned" against
the reference binary; these tests pin the pieces that can be pinned (linear algebra against
numpy, the LM's fixed point against the fixture's known true pose, the faithful mode's
no-update semantics, MO:1539-1545).
"""
import os

import numpy as np
import pytest


import oracle_py
from llsr import _abi

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mo_map_vlp16.npz")


def _spd(rng, n, cond=1e3):
    Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
    ev = np.geomspace(1.0, cond, n) * rng.uniform(0.5, 2.0)
    return (Q * ev) @ Q.T


@pytest.mark.parametrize("n", [3, 6])
def test_eig_matches_numpy(n):
    rng = np.random.default_rng(n)
    for _ in range(200):
        A = _spd(rng, n).astype(np.float32)
        A = (A + A.T) / 2
        ev, V = oracle_py.eig(A)
        ref = np.linalg.eigvalsh(A.astype(np.float64))
        assert np.all(np.diff(ev) >= 0), "Eigen sorts ascending"
        np.testing.assert_allclose(ev, ref, rtol=2e-5, atol=2e-5 * np.abs(ref).max())
        np.testing.assert_allclose(V.T @ V, np.eye(n), atol=5e-6 * n)
        resid = A @ V - V * ev
        assert np.abs(resid).max() <= 5e-6 * np.abs(ref).max() * n


def test_eig3_degenerate_and_diagonal():
    # repeated eigenvalues / already-diagonal input: the restatement must still converge
    for A in (np.eye(3), np.diag([3.0, 1.0, 2.0]), np.ones((3, 3)), np.zeros((3, 3))):
        ev, V = oracle_py.eig(A.astype(np.float32))
        np.testing.assert_allclose(ev, np.linalg.eigvalsh(A), atol=1e-6)


def test_qr_solve_5x3_least_squares():
    rng = np.random.default_rng(5)
    for _ in range(200):
        A = rng.normal(size=(5, 3)).astype(np.float32)
        b = rng.normal(size=5).astype(np.float32)
        x = oracle_py.qr_solve(A, b)
        ref = np.linalg.lstsq(A.astype(np.float64), b.astype(np.float64), rcond=None)[0]
        np.testing.assert_allclose(x, ref, rtol=1e-4, atol=1e-5)


def test_qr_solve_6x6():
    rng = np.random.default_rng(6)
    for _ in range(200):
        A = _spd(rng, 6, cond=1e2).astype(np.float32)
        b = rng.normal(size=6).astype(np.float32)
        x = oracle_py.qr_solve(A, b)
        np.testing.assert_allclose(x, np.linalg.solve(A.astype(np.float64), b), rtol=1e-4, atol=1e-5)


@pytest.fixture(scope="module")
def fix():
    return np.load(FIX)


def _run(fix, i, mode):
    cfg = _abi.config_for("vlp16")
    cfg.mode = mode
    return oracle_py.scan2map(cfg, fix[f"q{i}_corner"], fix[f"q{i}_surf"], fix["corner_map"],
                              fix["surf_map"], fix[f"q{i}_init"])


def test_fixture_shape(fix):
    assert len(fix["corner_map"]) + len(fix["surf_map"]) > 70000
    for i in range(int(fix["n_queries"])):
        assert len(fix[f"q{i}_corner"]) > 100 and len(fix[f"q{i}_surf"]) > 1000


@pytest.mark.parametrize("i", [0, 1, 2, 3])
def test_lm_applied_recovers_pose(fix, i):
    r = _run(fix, i, _abi.LLSR_MODE_LM_APPLIED)
    assert r["converged"] and not r["degenerate"]
    assert r["iterations"] < 20
    assert np.abs(r["pose"] - fix[f"q{i}_true"]).max() < 0.02
    assert r["n_corner_corr"] > 50 and r["n_surf_corr"] > 1000


def test_faithful_mode_never_updates(fix):
    # MO:1539-1545: the transformTobeMapped update is commented out in the reference, so the
    # pose is untouched and every iteration re-derives the same step until iterCountThres
    r0 = _run(fix, 0, _abi.LLSR_MODE_FAITHFUL)
    r1 = _run(fix, 0, _abi.LLSR_MODE_LM_APPLIED)
    np.testing.assert_array_equal(r0["pose"], fix["q0_init"])
    assert r0["iterations"] == 200 and not r0["converged"]
    np.testing.assert_array_equal(r0["matX0"], r1["matX0"])  # same first step


def test_empty_map_is_a_no_op(fix):
    # scan2MapOptimization's guard (MO:1573): too few map points -> no optimisation
    cfg = _abi.config_for("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    r = oracle_py.scan2map(cfg, fix["q0_corner"], fix["q0_surf"], fix["corner_map"][:10],
                           fix["surf_map"], fix["q0_init"])
    np.testing.assert_array_equal(r["pose"], fix["q0_init"])
    assert r["iterations"] == 0


def _need_ref():
    if oracle_py.ref_lib() is None:
        pytest.skip("oracle/_ref/libref_mo.so not built (needs /root/reference)")


@pytest.mark.parametrize("which", ["corner_map", "surf_map"])
def test_grid_knn_equals_reference_kdtree(fix, which):
    """The restatement's 1 m grid == the reference's nanoflann kd-tree (nanoflann_pcl.h:
    SO3_Adaptor over L2_Simple, leaf 10), index for index and bit for bit in d^2."""
    _need_ref()
    m = fix[which]
    rng = np.random.default_rng(11)
    q = m[rng.integers(0, len(m), 20000)].copy()
    q[:, :3] += rng.normal(0.0, 0.3, (len(q), 3)).astype(np.float32)
    ig, dg = oracle_py.knn5(m, q, "grid")
    ik, dk = oracle_py.knn5(m, q, "kdtree")
    assert (ig[:, 0] >= 0).sum() > 10000
    np.testing.assert_array_equal(ig, ik)
    np.testing.assert_array_equal(dg, dk)


@pytest.mark.parametrize("mode", [_abi.LLSR_MODE_LM_APPLIED, _abi.LLSR_MODE_FAITHFUL])
def test_scan2map_grid_equals_reference_kdtree(fix, mode):
    _need_ref()
    cfg = _abi.config_for("vlp16")
    cfg.mode = mode
    args = (fix["q1_corner"], fix["q1_surf"], fix["corner_map"], fix["surf_map"], fix["q1_init"])
    rg = oracle_py.scan2map(cfg, *args)
    rk = oracle_py.scan2map(cfg, *args, knn="kdtree")
    for k in rg:
        if k != "ms":
            np.testing.assert_array_equal(np.asarray(rg[k]), np.asarray(rk[k]), err_msg=k)
