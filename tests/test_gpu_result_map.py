"""GPU parity on the reference's own recorded mapping run (Result/0318_test ->
tests/golden/result_0318.npz; tests/_result_map.py builds the problems): real-sensor map geometry
for the scan-to-map LM in both modes (MO:1269-1570), the key-pose VoxelGrid and the whole
extractSurroundingKeyFrames (MO:1096-1232) over the recorded trajectory. Bar: bit-exact against
the oracle, whose kNN and radius search equal the reference's own nanoflann on the same data
(tests/test_result_fixture.py); the faithful mode runs the 200 iterations MapIterTimes.txt
records for every frame of that run."""
import ctypes

import numpy as np
import pytest

import _result_map as R
import oracle_py
from llsr import LocalMap, Pipeline, _abi, default_config

pytestmark = pytest.mark.gpu
KEYS = ("pose", "matX0", "min_lambda", "cf_mean", "iterations", "converged", "degenerate",
        "n_corner_corr", "n_surf_corr")


@pytest.fixture(scope="module")
def z():
    return R.load()


@pytest.fixture(scope="module")
def probs(z):
    return R.scan2map_problems(z)


def _cfg(mode):
    cfg = default_config("vlp16")
    cfg.mode = mode
    return cfg


@pytest.mark.parametrize("mode", [_abi.LLSR_MODE_LM_APPLIED, _abi.LLSR_MODE_FAITHFUL])
def test_scan2map_on_recorded_map(require_gpu, z, probs, mode):
    cfg = _cfg(mode)
    pipe = Pipeline(cfg)
    errs = []
    use = probs if mode == _abi.LLSR_MODE_LM_APPLIED else probs[:2]
    for k, (cq, sq, cm, sm, p0, true) in enumerate(use):
        g = pipe.scan2map(cq, sq, cm, sm, p0)
        o = oracle_py.scan2map(cfg, cq, sq, cm, sm, p0)
        errs += [f"problem {k}: {key} {g[key]} vs {o[key]}" for key in KEYS
                 if not np.array_equal(np.asarray(g[key]), np.asarray(o[key]))]
        if mode == _abi.LLSR_MODE_FAITHFUL:
            assert g["iterations"] == int(z["map_iter_times"][0]) == 200  # MapIterTimes.txt
        else:
            assert np.abs(g["pose"] - true).max() < 0.03
    pipe.close()
    assert not errs, "\n".join(errs)


@pytest.mark.parametrize("mode", [_abi.LLSR_MODE_LM_APPLIED, _abi.LLSR_MODE_FAITHFUL])
def test_scan2map_on_recorded_map_vs_reference_kdtree(require_gpu, probs, mode):
    """The HIP scan-to-map against the MO restatement running over the REFERENCE's own nanoflann
    kd-tree (oracle/_ref, compiled from the reference's nanoflann.hpp; it travels to the GPU box
    prebuilt) on the recorded real-sensor map: every recorded problem bit-exact, so on this geometry
    the device's cell-grid kNN-5 (ties by index) and nanoflann's (ties in tree order) agree."""
    if oracle_py.ref_lib() is None:
        pytest.skip("oracle/_ref/libref_mo.so not built")
    cfg = _cfg(mode)
    pipe = Pipeline(cfg)
    errs = []
    use = probs if mode == _abi.LLSR_MODE_LM_APPLIED else probs[:2]
    for k, (cq, sq, cm, sm, p0, _) in enumerate(use):
        g = pipe.scan2map(cq, sq, cm, sm, p0)
        o = oracle_py.scan2map(cfg, cq, sq, cm, sm, p0, knn="kdtree")
        errs += [f"problem {k}: {key} {g[key]} vs {o[key]}" for key in KEYS
                 if not np.array_equal(np.asarray(g[key]), np.asarray(o[key]))]
    pipe.close()
    assert not errs, "\n".join(errs)


def test_scan2map_batch_on_recorded_map(require_gpu, probs):
    """The five recorded-map problems as one device batch (llsr_scan2map_batch), lm_applied."""
    import torch
    cfg = _cfg(_abi.LLSR_MODE_LM_APPLIED)
    P = len(probs)

    def pack(k):
        arrs = [np.ascontiguousarray(pr[k], np.float32) for pr in probs]
        off = np.zeros(P + 1, np.int64)
        off[1:] = np.cumsum([len(a) for a in arrs])
        return torch.from_numpy(np.concatenate(arrs)).cuda(), torch.from_numpy(off).cuda()

    (cq, cqo), (sq, sqo), (cm, cmo), (sm, smo) = (pack(k) for k in range(4))
    pose = torch.from_numpy(np.stack([pr[4] for pr in probs])).cuda()
    n = ctypes.sizeof(_abi.LmReport)
    rep = torch.zeros(P * n // 4, dtype=torch.float32, device="cuda")
    pipe = Pipeline(cfg)
    pipe.scan2map_reserve(P, *(max(len(pr[k]) for pr in probs) for k in (2, 3, 0, 1)))
    torch.cuda.synchronize()
    pipe.scan2map_batch(dict(corner_q=cq.data_ptr(), corner_q_off=cqo.data_ptr(), surf_q=sq.data_ptr(),
                             surf_q_off=sqo.data_ptr(), corner_map=cm.data_ptr(), corner_map_off=cmo.data_ptr(),
                             surf_map=sm.data_ptr(), surf_map_off=smo.data_ptr(), pose=pose.data_ptr(),
                             report=rep.data_ptr()), P)
    torch.cuda.synchronize()
    poses, raw = pose.cpu().numpy(), rep.cpu().numpy().tobytes()
    pipe.close()
    for p, pr in enumerate(probs):
        o = oracle_py.scan2map(cfg, *pr[:5])
        r = _abi.LmReport.from_buffer_copy(raw[p * n:(p + 1) * n])
        np.testing.assert_array_equal(poses[p], o["pose"])
        assert (r.iterations, r.converged, r.n_corner_corr, r.n_surf_corr) == \
            (o["iterations"], o["converged"], o["n_corner_corr"], o["n_surf_corr"]), p


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_keypose_voxel_grid_on_recorded_trajectory(require_gpu, z):
    """downSizeFilterSurroundingKeyPoses (VoxelGrid 1.0, MO:99, 1162-1166) of the recorded key
    poses (x, y, z, index), and the 0.2 / 0.4 VoxelGrids of the recorded maps: bit-exact."""
    key = z["key_poses"]
    poses4 = np.concatenate([key[:, :3], np.arange(len(key), dtype=np.float32)[:, None]], axis=1)
    m = LocalMap(0)
    clouds = [poses4, z["corner_map"], z["surf_map"]]
    leaves = [1.0, 0.2, 0.4]
    outs = m.voxel_grid(clouds, leaves)
    for c, leaf, g in zip(clouds, leaves, outs):
        ref = oracle_py.voxel_grid(c, leaf)
        got = g.detach().cpu().numpy()
        assert got.shape == ref.shape and np.array_equal(_bits(got), _bits(ref)), leaf
    m.close()


def test_extract_surrounding_keyframes_on_recorded_trajectory(require_gpu, z):
    """The whole extractSurroundingKeyFrames (radius branch, MO:1152-1232) while the recorded run's
    723 keyframes are added in order: the recorded key poses, each keyframe's share of the recorded
    maps (tests/_result_map.keyframes); keyframe ids, raw sizes and both local maps bit-exact."""
    frames = R.keyframes(z)
    m = LocalMap(0)
    om = oracle_py.OracleMap(radius=50.0)
    checked = 0
    for k, (pose, c, s, o) in enumerate(frames):
        assert m.add_keyframe(pose, c, s, o) == k
        om.add_keyframe(pose, c, s, o)
        if k % 60 != 5 and k != len(frames) - 1:
            continue
        pos = pose[:3] + np.float32(0.1)
        gc, gs, rep = m.extract(pos)
        rc, rs, ids, orep = om.extract(pos)
        assert m.keyframe_ids().tolist() == ids.tolist(), k
        for key in ("n_in_radius", "n_poses_ds", "n_keyframes", "n_corner_map", "n_surf_map"):
            assert rep[key] == orep[key], (k, key)
        assert np.array_equal(_bits(gc.detach().cpu().numpy()), _bits(rc)), k
        assert np.array_equal(_bits(gs.detach().cpu().numpy()), _bits(rs)), k
        checked += 1
    assert checked >= 12 and orep["n_in_radius"] == len(frames)
    m.close()
