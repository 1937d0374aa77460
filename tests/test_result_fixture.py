"""CPU: the reference's own recorded mapping run (Result/0318_test -> tests/golden/result_0318.npz,
tests/golden/make_result_fixture.py) pins what it can of the oracle: the faithful mode's iteration
count (MapIterTimes.txt = 200 on every frame), the kNN and the key-pose radius search against the
reference's own nanoflann.hpp (oracle/_ref) on real-sensor geometry, and the scan-to-map LM on the
recorded map with both kNN implementations. The GPU side of the same problems is
tests/test_gpu_result_map.py."""
import numpy as np
import pytest

import _result_map as R
import oracle_py
from llsr import _abi


@pytest.fixture(scope="module")
def z():
    return R.load()


@pytest.fixture(scope="module")
def probs(z):
    return R.scan2map_problems(z)


def _need_ref():
    if oracle_py.ref_lib() is None:
        pytest.skip("oracle/_ref/libref_mo.so not built (needs /root/reference)")


def _cfg(mode):
    cfg = _abi.config_for("vlp16")
    cfg.mode = mode
    return cfg


def test_fixture_matches_the_recorded_files(z):
    key = z["key_poses"]
    assert len(z["corner_map"]) == 84644 and len(z["surf_map"]) == 6014 and len(key) == 723
    # trajectory.pcd and pose.txt describe the same key positions (pose.txt: z, x, y columns)
    assert np.abs(key[:, :3] - z["pose_txt_xyz"]).max() < 1e-6
    np.testing.assert_array_equal(z["traj_index"], np.arange(len(key)))  # intensity = index
    # MapIterTimes.txt: one scan2MapOptimization per frame after the first, 200 iterations each
    assert len(z["map_iter_times"]) == len(key) - 1
    assert set(z["map_iter_times"].tolist()) == {200.0}


def test_faithful_mode_runs_the_recorded_200_iterations(z, probs):
    """The recorded run's MapIterTimes (200 on every frame) is the faithful mode's fixed count: the
    pose update is commented out (MO:1539-1545), so the LM never converges before iterCountThres."""
    cfg = _cfg(_abi.LLSR_MODE_FAITHFUL)
    assert cfg.iterCountThres == int(z["map_iter_times"].max())
    cq, sq, cm, sm, p0, _ = probs[0]
    o = oracle_py.scan2map(cfg, cq, sq, cm, sm, p0)
    assert o["iterations"] == 200 and not o["converged"]
    np.testing.assert_array_equal(o["pose"], p0)


def test_lm_applied_recovers_recorded_key_poses(probs):
    cfg = _cfg(_abi.LLSR_MODE_LM_APPLIED)
    for cq, sq, cm, sm, p0, true in probs:
        o = oracle_py.scan2map(cfg, cq, sq, cm, sm, p0)
        assert o["converged"] and not o["degenerate"]
        assert o["n_corner_corr"] > 300 and o["n_surf_corr"] > 1000
        assert np.abs(o["pose"] - true).max() < 0.03


@pytest.mark.parametrize("which", ["corner_raw", "corner_ds", "surf"])
def test_knn5_equals_reference_kdtree_on_recorded_map(z, probs, which):
    """kNN-5 (nanoflann KdTreeFLANN, MO:1275-1276, 1387) on the recorded maps: the restatement's
    grid == the reference's own nanoflann.hpp, index for index and bit for bit in d^2."""
    _need_ref()
    m = {"corner_raw": z["corner_map"], "corner_ds": probs[0][2], "surf": z["surf_map"]}[which]
    rng = np.random.default_rng(3)
    q = m[rng.integers(0, len(m), 20000)].copy()
    q[:, :3] += rng.normal(0.0, 0.2, (len(q), 3)).astype(np.float32)
    ig, dg = oracle_py.knn5(m, q, "grid")
    ik, dk = oracle_py.knn5(m, q, "kdtree")
    assert (ig[:, 4] >= 0).sum() > 15000  # -1 rows: the 5th neighbour is 1 m or farther (MO:1280)
    np.testing.assert_array_equal(ig, ik)
    np.testing.assert_array_equal(dg, dk)


@pytest.mark.parametrize("radius", [50.0, 2.0, 0.5])
def test_keypose_radius_equals_reference_kdtree_on_recorded_trajectory(z, radius):
    """radiusSearch over cloudKeyPoses3D (MO:1155-1157) at every recorded key position: brute force
    == the reference's nanoflann; 50 m is the config's radius (every key pose of this indoor run is
    inside it), the smaller radii make the comparison discriminate."""
    _need_ref()
    key = z["key_poses"]
    poses4 = np.concatenate([key[:, :3], np.arange(len(key), dtype=np.float32)[:, None]], axis=1)
    sizes = []
    for k in range(0, len(key), 7):
        a = oracle_py.keypose_radius(poses4, key[k, :3], radius)
        b = oracle_py.keypose_radius(poses4, key[k, :3], radius, knn="kdtree")
        np.testing.assert_array_equal(a, b)
        sizes.append(len(a))
    assert min(sizes) >= 1 and (radius == 50.0) == (min(sizes) == len(key))


@pytest.mark.parametrize("mode", [_abi.LLSR_MODE_LM_APPLIED, _abi.LLSR_MODE_FAITHFUL])
def test_scan2map_grid_equals_reference_kdtree_on_recorded_map(probs, mode):
    _need_ref()
    cfg = _cfg(mode)
    cq, sq, cm, sm, p0, _ = probs[1]
    rg = oracle_py.scan2map(cfg, cq, sq, cm, sm, p0)
    rk = oracle_py.scan2map(cfg, cq, sq, cm, sm, p0, knn="kdtree")
    for k in rg:
        if k != "ms":
            np.testing.assert_array_equal(np.asarray(rg[k]), np.asarray(rk[k]), err_msg=k)
