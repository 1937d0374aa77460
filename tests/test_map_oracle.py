"""CPU tests of the local-map restatement (oracle/oracle_map.cpp, oracle/oracle_voxel.h):
MapOptimization::extractSurroundingKeyFrames (MO:1096-1232) and pcl::VoxelGrid.

Pinning: the key-pose radius search is checked against the reference's own nanoflann kd-tree
(oracle/_ref, built from LeGO-LOAM/include/lego_loam/nanoflann.hpp by path). PCL is not in the
reference or the image: the VoxelGrid restatement follows PCL 1.10's published applyFilter and is
checked here against an independent scalar statement of the same algorithm (parity with PCL itself
unpinned). The surroundingExistingKeyPosesID bookkeeping is checked against a second, list-based
statement of MO:1169-1222."""
import numpy as np
import pytest

import oracle_py
from llsr import synth


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _vg_scalar(pts, leaf):
    """Independent statement of PCL VoxelGrid with a stable sort (sum in input order)."""
    pts = np.asarray(pts, np.float32)
    if len(pts) == 0:
        return pts.reshape(0, 4)
    inv = np.float32(1.0) / np.float32(leaf)
    mn, mx = pts[:, :3].min(0), pts[:, :3].max(0)
    d = [int(np.float32((mx[a] - mn[a]) * inv)) + 1 for a in range(3)]
    if d[0] * d[1] * d[2] > 2**31 - 1:
        return pts.copy()
    minb = [int(np.floor(np.float32(mn[a] * inv))) for a in range(3)]
    maxb = [int(np.floor(np.float32(mx[a] * inv))) for a in range(3)]
    div = [maxb[a] - minb[a] + 1 for a in range(3)]
    ijk = [(np.floor(pts[:, a] * inv) - np.float32(minb[a])).astype(np.int64) for a in range(3)]
    idx = (ijk[0] + ijk[1] * div[0] + ijk[2] * div[0] * div[1]) & 0xFFFFFFFF
    order = np.argsort(idx, kind="stable")
    out = []
    k = 0
    while k < len(order):
        e = k
        while e < len(order) and idx[order[e]] == idx[order[k]]:
            e += 1
        s = [np.float32(0)] * 4
        for q in order[k:e]:
            for a in range(4):
                s[a] = np.float32(s[a] + pts[q, a])
        n = np.float32(e - k)
        out.append([np.float32(v / n) for v in s])
        k = e
    return np.array(out, np.float32)


def test_voxel_grid_matches_scalar_statement():
    rng = np.random.default_rng(3)
    pts = np.concatenate([rng.normal(0, 2, (1500, 4)), rng.uniform(-6, 6, (500, 4))]).astype(np.float32)
    for leaf in (0.2, 0.4, 1.0):
        ref = _vg_scalar(pts, leaf)
        got = oracle_py.voxel_grid(pts, leaf, stable=True)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        pcl = oracle_py.voxel_grid(pts, leaf)
        assert pcl.shape == ref.shape
        np.testing.assert_allclose(pcl, ref, rtol=1e-6, atol=1e-5)


def test_voxel_grid_edge_cases():
    assert oracle_py.voxel_grid(np.zeros((0, 4), np.float32), 0.2).shape == (0, 4)
    one = np.array([[1.25, -3.5, 7.0, 4.0]], np.float32)
    assert np.array_equal(oracle_py.voxel_grid(one, 0.2), one)
    same = np.repeat(one, 17, axis=0)
    assert np.array_equal(oracle_py.voxel_grid(same, 0.4, stable=True), one)
    # (max - min) / leaf product over INT32_MAX: PCL returns the input unchanged
    rng = np.random.default_rng(5)
    wide = rng.uniform(-5e3, 5e3, (300, 4)).astype(np.float32)
    assert np.array_equal(oracle_py.voxel_grid(wide, 0.2), wide)


def test_keypose_radius_matches_reference_kdtree():
    if oracle_py.ref_lib() is None:
        pytest.skip("oracle/_ref not built (no /root/reference and no prebuilt copy)")
    rng = np.random.default_rng(11)
    poses = np.zeros((600, 4), np.float32)
    poses[:, :3] = rng.uniform(-90, 90, (600, 3)).astype(np.float32)
    poses[:, 3] = np.arange(600, dtype=np.float32)
    # exact-boundary poses: d^2 == 2500 is outside (RadiusResultSet keeps dist < radius)
    poses[:4, :3] = [[50, 0, 0], [0, -50, 0], [0, 0, 50], [30, 40, 0]]
    for q in [np.zeros(3, np.float32)] + [rng.uniform(-60, 60, 3).astype(np.float32) for _ in range(25)]:
        a = oracle_py.keypose_radius(poses, q, 50.0)
        b = oracle_py.keypose_radius(poses, q, 50.0, knn="kdtree")
        assert np.array_equal(a, b)
    assert not {0, 1, 2, 3} & set(oracle_py.keypose_radius(poses, np.zeros(3, np.float32), 50.0).tolist())


def test_extract_keyframe_list_semantics():
    """surroundingExistingKeyPosesID after each call equals a direct statement of MO:1169-1222."""
    frames = synth.make_keyframes(48, seed=2, corner=20, surf=40, outlier=10)
    om = oracle_py.OracleMap(radius=50.0)
    existing = []
    saw_drop = saw_avg = False
    for k, (pose, c, s, o) in enumerate(frames):
        om.add_keyframe(pose, c, s, o)
        pos = pose[:3] + np.float32(0.3)
        _, _, ids, rep = om.extract(pos)
        P = np.array([[*f[0][:3], i] for i, f in enumerate(frames[:k + 1])], np.float32)
        sel = oracle_py.keypose_radius(P, pos, 50.0)
        ds = oracle_py.voxel_grid(P[sel], 1.0)
        ds_ids = [int(v) for v in ds[:, 3]]
        saw_avg |= any(float(v) != int(v) for v in ds[:, 3])
        kept = [i for i in existing if i in ds_ids]
        saw_drop |= len(kept) < len(existing)
        existing = kept + [d for i, d in enumerate(ds_ids) if d not in kept and d not in ds_ids[:i]]
        assert ids.tolist() == existing
        assert rep["n_in_radius"] == len(sel) and rep["n_poses_ds"] == len(ds)
        assert rep["n_corner_map"] == sum(len(frames[i][1]) for i in existing)
        assert rep["n_surf_map"] == sum(len(frames[i][2]) + len(frames[i][3]) for i in existing)
    assert saw_drop and saw_avg, "the synthetic path must exercise list removal and index averaging"


@pytest.mark.parametrize("search_num", [1, 4, 50])
def test_extract_loop_closure_queue(search_num):
    """enable_loop_closure (CFG:91, 159): the local map is the recent-keyframe queue of MO:1099-1151.
    Checked against a list statement: while the queue is shorter than search_num it holds the
    newest min(K, search_num) keyframes (rebuilt every call); once full, one pop-oldest / push-newest
    per new keyframe; a repeated call without a new keyframe keeps it (latestFrameID, MO:1126). The
    local map is the VoxelGrid of the queue's transformed clouds in queue order, surf + outlier per
    keyframe (MO:1147-1151, 1224-1231)."""
    frames = synth.make_keyframes(12, seed=5, corner=30, surf=60, outlier=15)
    om = oracle_py.OracleMap(loop_closure=True, search_num=search_num)
    radius = oracle_py.OracleMap(radius=1e-3)  # a radius branch that would select nothing near
    q = []
    latest = 0
    for k, (pose, c, s, o) in enumerate(frames):
        om.add_keyframe(pose, c, s, o)
        radius.add_keyframe(pose, c, s, o)
        for rep_call in range(2 if k in (3, 7) else 1):
            K = k + 1
            if len(q) < search_num:
                q = list(range(max(0, K - search_num), K))
            elif latest != K - 1:
                q = q[1:] + [K - 1]
                latest = K - 1
            cmap, smap, ids, rep = om.extract(np.full(3, 1e4, np.float32))  # position unused
            assert ids.tolist() == q, (k, rep_call)
            assert rep["n_in_radius"] == 0 and rep["n_poses_ds"] == 0 and rep["n_keyframes"] == len(q)
            assert rep["n_corner_map"] == sum(len(frames[i][1]) for i in q)
            assert rep["n_surf_map"] == sum(len(frames[i][2]) + len(frames[i][3]) for i in q)
            # the same keyframes through the radius branch's transform + VoxelGrid path
            cm = [oracle_py.transform_keyframe(frames[i][0], frames[i][1]) for i in q]
            sm = [x for i in q for x in (oracle_py.transform_keyframe(frames[i][0], frames[i][2]),
                                         oracle_py.transform_keyframe(frames[i][0], frames[i][3]))]
            assert np.array_equal(_bits(cmap), _bits(oracle_py.voxel_grid(np.concatenate(cm), 0.2)))
            assert np.array_equal(_bits(smap), _bits(oracle_py.voxel_grid(np.concatenate(sm), 0.4)))
    _, _, ids_r, _ = radius.extract(np.full(3, 1e4, np.float32))
    assert len(ids_r) == 0
