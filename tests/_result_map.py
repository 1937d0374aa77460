"""Problems built on the reference's own recorded map (tests/golden/result_0318.npz, converted from
Result/0318_test by tests/golden/make_result_fixture.py): real-sensor geometry for the scan-to-map
LM (MO:1269-1570), the kNN (nanoflann), the key-pose radius search and the local map
(extractSurroundingKeyFrames, MO:1096-1232).

* Scan-to-map: the local map is the recorded corner map through VoxelGrid 0.2 (downSizeFilterCorner,
  MO:92) and the recorded surf map (already VoxelGrid 0.4); the queries of key pose k are map points
  around its position with 1 cm noise, moved into the keyframe's own frame by the inverse of
  transformPointCloud (MO:671-701) at that key pose; the optimiser starts from the key pose
  (transformTobeMapped = roll, pitch, yaw, x, y, z) perturbed by a seeded (0.05 rad, 0.2 m).
* Local map: the recorded clouds partitioned into per-keyframe clouds (each map point to its
  nearest key position), in the keyframe's own frame, with the recorded key poses.
"""
import os

import numpy as np

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "result_0318.npz")


def load():
    return np.load(FIX)


def _rot(pose6):
    """transformPointCloud's rotation (MO:681-696): p' = Ry(pitch) Rx(roll) Rz(yaw) p + t."""
    roll, pitch, yaw = (float(a) for a in pose6[3:6])
    cy, sy, cr, sr, cp, sp = np.cos(yaw), np.sin(yaw), np.cos(roll), np.sin(roll), np.cos(pitch), np.sin(pitch)
    rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    return ry @ rx @ rz


def to_key_frame(pose6, pts):
    """The inverse of transformPointCloud at key pose `pose6` (x, y, z, roll, pitch, yaw), float64."""
    out = np.array(pts, np.float32, copy=True)
    p = pts[:, :3].astype(np.float64) - np.asarray(pose6[:3], np.float64)
    out[:, :3] = (p @ _rot(pose6)).astype(np.float32)  # R^T p, row-vector form
    return out


def scan2map_problems(z, keys=(40, 200, 380, 560, 700), n_corner=1200, n_surf=1500, seed=5):
    """[(corner_q, surf_q, corner_map, surf_map, pose0, pose_true)] on the recorded map."""
    import oracle_py
    rng = np.random.default_rng(seed)
    cmap = oracle_py.voxel_grid(z["corner_map"], 0.2)
    smap = np.ascontiguousarray(z["surf_map"])
    out = []
    for k in keys:
        kp = z["key_poses"][k]
        pos = kp[:3].astype(np.float64)
        qs = []
        for src, r, n in ((cmap, 6.0, n_corner), (smap, 8.0, n_surf)):
            near = np.flatnonzero(((src[:, :3] - pos) ** 2).sum(1) < r * r)
            pick = src[rng.choice(near, size=min(n, len(near)), replace=False)].copy()
            pick[:, :3] += rng.normal(0.0, 0.01, (len(pick), 3)).astype(np.float32)
            qs.append(to_key_frame(kp, pick))
        true = np.array([kp[3], kp[4], kp[5], kp[0], kp[1], kp[2]], np.float32)
        pose0 = true + np.concatenate([rng.uniform(-0.05, 0.05, 3), rng.uniform(-0.2, 0.2, 3)]).astype(np.float32)
        out.append((qs[0], qs[1], cmap, smap, pose0, true))
    return out


def keyframes(z):
    """[(pose6, corner, surf, outlier)] per recorded key pose: the recorded clouds split by nearest
    key position and moved into each keyframe's frame (outlier clouds empty)."""
    from scipy.spatial import cKDTree
    key = z["key_poses"]
    tree = cKDTree(key[:, :3].astype(np.float64))
    parts = []
    for cloud in (z["corner_map"], z["surf_map"]):
        _, owner = tree.query(cloud[:, :3].astype(np.float64))
        order = np.argsort(owner, kind="stable")  # each keyframe's points in recorded order
        parts.append(np.split(order, np.searchsorted(owner[order], np.arange(1, len(key)))))
    empty = np.zeros((0, 4), np.float32)
    return [(key[k].copy(), to_key_frame(key[k], z["corner_map"][parts[0][k]]),
             to_key_frame(key[k], z["surf_map"][parts[1][k]]), empty) for k in range(len(key))]
