"""Seeded synthetic lidar scans for parity tests and bench.py.

A ray-cast street scene — ground plane at z = -1.3 m (the ELEVATION prior of
imageProjection.cpp:674-675), building facades with recessed windows and pillars, parked
cars, poles, tree trunks — sampled with the beam layout of a VLP-16 (16 rings at
-15 + 2 r deg, 1800 azimuth bins) or an HDL-64E (64 rings evenly over -24.8..+2.0 deg,
2048 bins). Every beam points at its range-image bin centre (IMAGE row value r + 0.05 / r +
0.235, column value an integer), so asinf/round in projectPointCloud (IP:313-323) never sit
near a truncation boundary. Points come in Velodyne order (azimuth-major, clockwise from the
rear; lasers in firing order), range noise N(0, 1 cm), 2 % dropout -> NaN, misses -> NaN.

Ground inside 10 m is an exact plane plus 1 cm noise and no obstacle base sits within
0.4-0.6 m of it, so PCL's RANSAC (IP:716-721) returns the same inlier set for any sample
(checked by tests/test_oracle.py::test_ransac_seed_independent).
"""
from __future__ import annotations

import numpy as np

VLP16 = "vlp16"
HDL64E = "hdl64e"

_VLP16_FIRING = np.array([-15, 1, -13, 3, -11, 5, -9, 7, -7, 9, -5, 11, -3, 13, -1, 15], dtype=np.float64)


def beam_layout(lidar: str):
    """Return (elevations_deg in firing order, num_columns)."""
    if lidar == VLP16:
        return _VLP16_FIRING.copy(), 1800
    if lidar == HDL64E:
        res = (2.0 - (-24.8)) / 63.0
        elev = -24.8 + res * np.arange(64, dtype=np.float64)
        # upper / lower block interleave like the HDL-64E's two laser blocks
        order = np.stack([np.arange(32, 64), np.arange(0, 32)], axis=1).reshape(-1)
        return elev[order], 2048
    raise ValueError(lidar)


class _Scene:
    def __init__(self, rng: np.random.Generator, ground_ramp: tuple[float, float] | None = None):
        # ground_ramp = (x0, slope): beyond x = x0 the ground rises with this slope (a second plane
        # the near-ground RANSAC can lock onto, tests/test_gpu_features_ties.py)
        self.ramp = ground_ramp
        boxes = []  # (xmin, xmax, ymin, ymax, zmin, zmax)
        # facades: left y in [9, 12], right y in [-14, -11], long along x
        for side, y0, y1 in ((1, 9.0, 12.0), (-1, -14.0, -11.0)):
            x = -70.0
            while x < 90.0:
                w = rng.uniform(8.0, 18.0)
                gap = rng.uniform(0.0, 4.0)
                setback = rng.uniform(0.0, 1.5) * side
                boxes.append((x, x + w, y0 + setback, y1 + setback, -1.3, rng.uniform(6.0, 15.0)))
                # pillars sticking out of the facade
                for px in np.arange(x + 1.0, x + w - 0.5, rng.uniform(2.5, 4.5)):
                    face = (y0 + setback) if side > 0 else (y1 + setback)
                    if side > 0:
                        boxes.append((px, px + 0.4, face - 0.35, face, -1.3, 4.0))
                    else:
                        boxes.append((px, px + 0.4, face, face + 0.35, -1.3, 4.0))
                x += w + gap
        # parked cars along both curbs
        for side in (1, -1):
            x = -60.0 + rng.uniform(0, 5)
            while x < 80.0:
                L, Wd, Hc = rng.uniform(3.8, 5.0), rng.uniform(1.7, 2.0), rng.uniform(1.3, 1.8)
                yc = side * rng.uniform(5.0, 6.0)
                if abs(x) > 4.0 or abs(yc) > 5.0:
                    boxes.append((x, x + L, yc - Wd / 2, yc + Wd / 2, -1.3 + 0.25, -1.3 + Hc))
                x += L + rng.uniform(1.5, 7.0)
        # street furniture: bins / boxes
        for _ in range(10):
            cx, cy = rng.uniform(-40, 60), rng.choice([-1, 1]) * rng.uniform(6.8, 8.2)
            s = rng.uniform(0.5, 1.2)
            boxes.append((cx, cx + s, cy, cy + s, -1.3, -1.3 + rng.uniform(0.9, 1.6)))
        self.boxes = np.array(boxes, dtype=np.float64)
        cyl = []  # (cx, cy, radius, zmin, zmax)
        for side in (1, -1):
            for x in np.arange(-60.0, 80.0, rng.uniform(10.0, 14.0)):
                cyl.append((x + rng.uniform(-1, 1), side * rng.uniform(7.0, 7.6), rng.uniform(0.1, 0.2), -1.3, rng.uniform(4.0, 7.0)))
            for x in np.arange(-55.0, 80.0, rng.uniform(14.0, 20.0)):  # tree trunks
                cyl.append((x + rng.uniform(-2, 2), side * rng.uniform(7.8, 8.6), rng.uniform(0.2, 0.35), -1.3, 3.0))
        self.cyl = np.array(cyl, dtype=np.float64)
        self.ground_z = -1.3

    def cast(self, o: np.ndarray, d: np.ndarray, tmax: float) -> np.ndarray:
        """Nearest hit distance along unit rays d from origin o (inf = miss)."""
        t = np.full(d.shape[0], np.inf)
        dz = d[:, 2]
        with np.errstate(divide="ignore", invalid="ignore"):
            tg = (self.ground_z - o[2]) / dz
        if self.ramp is None:
            t = np.where((dz < 0) & (tg > 0), tg, t)
        else:
            x0, k = self.ramp
            flat_ok = (dz < 0) & (tg > 0) & (o[0] + tg * d[:, 0] <= x0)
            with np.errstate(divide="ignore", invalid="ignore"):  # z = ground_z + k (x - x0)
                tr = (self.ground_z + k * (o[0] - x0) - o[2]) / (dz - k * d[:, 0])
            ramp_ok = (tr > 0) & (o[0] + tr * d[:, 0] > x0)
            t = np.where(flat_ok, tg, t)
            t = np.where(ramp_ok & (tr < t), tr, t)
        inv = 1.0 / np.where(np.abs(d) < 1e-12, 1e-12, d)
        for b in self.boxes:
            t1 = (b[0::2] - o) * inv  # x/y/z mins
            t2 = (b[1::2] - o) * inv
            tn = np.minimum(t1, t2).max(axis=1)
            tf = np.maximum(t1, t2).min(axis=1)
            hit = (tf >= tn) & (tn > 0.05)
            t = np.where(hit & (tn < t), tn, t)
        dxy2 = d[:, 0] ** 2 + d[:, 1] ** 2
        for c in self.cyl:
            ox, oy = o[0] - c[0], o[1] - c[1]
            bq = ox * d[:, 0] + oy * d[:, 1]
            cq = ox * ox + oy * oy - c[2] * c[2]
            disc = bq * bq - dxy2 * cq
            with np.errstate(invalid="ignore", divide="ignore"):
                th = (-bq - np.sqrt(disc)) / dxy2
            z = o[2] + th * d[:, 2]
            hit = (disc > 0) & (th > 0.05) & (z >= c[3]) & (z <= c[4])
            t = np.where(hit & (th < t), th, t)
        t[t > tmax] = np.inf
        return t


def sensor_attitude(seed: int) -> np.ndarray:
    """The moving sensor's (dz, roll, pitch, yaw) for frame `seed` of its drive (radians / m).

    A vehicle on an uneven road: each DoF is a sum of two sinusoids over the frame index
    k = seed % 64 with phases drawn from the drive (scene) seed, amplitudes bounded by 5 cm in z,
    2 deg in roll and pitch and 3 deg in yaw. Consecutive frames differ by up to ~1.5 deg in roll /
    pitch and a few cm in z, which is what the scan-to-scan surf step solves for (pitch, roll and
    the vertical translation, featureAssociation.cpp:2001-2003): without it that step converges
    at its first iteration."""
    k = float(seed % 64)
    ph = np.random.default_rng(7700001 + seed // 64).uniform(0.0, 2.0 * np.pi, (4, 2))
    amp = np.array([0.05, np.deg2rad(2.0), np.deg2rad(2.0), np.deg2rad(3.0)])
    freq = np.array([[0.9, 2.3], [0.7, 1.9], [0.8, 2.1], [0.4, 1.3]])
    return amp * (0.6 * np.sin(freq[:, 0] * k + ph[:, 0]) + 0.4 * np.sin(freq[:, 1] * k + ph[:, 1]))


def _rot_zyx(roll: float, pitch: float, yaw: float) -> np.ndarray:
    cr, sr, cp, sp, cy, sy = np.cos(roll), np.sin(roll), np.cos(pitch), np.sin(pitch), np.cos(yaw), np.sin(yaw)
    rz = np.array([[cy, -sy, 0.0], [sy, cy, 0.0], [0.0, 0.0, 1.0]])
    ry = np.array([[cp, 0.0, sp], [0.0, 1.0, 0.0], [-sp, 0.0, cp]])
    rx = np.array([[1.0, 0.0, 0.0], [0.0, cr, -sr], [0.0, sr, cr]])
    return rz @ ry @ rx


def make_scan(seed: int, lidar: str = VLP16, dropout: float = 0.02, noise: float = 0.01,
              max_range: float = 100.0, origin_xy: tuple[float, float] | None = None,
              scene_id: int | None = None, ground_ramp: tuple[float, float] | None = None,
              motion: bool = False) -> np.ndarray:
    """One raw scan as float32 [N, 4] (x, y, z, intensity), N = rings * columns (NaNs kept).

    The sensor sits at (0.5 * (seed % 64), U(-0.5, 0.5), 0) of scene `seed // 64`; scan-to-map
    fixtures override both (`origin_xy`, `scene_id`) to place keyframes along one street. With
    `motion` the sensor also carries the drive's 6-DoF attitude (`sensor_attitude`): the rays are
    cast in the world from the tilted, yawed sensor and the points are returned in the sensor's own
    frame, so every beam still points at its range-image bin centre."""
    rng = np.random.default_rng(seed)
    scene_id = seed // 64 if scene_id is None else scene_id  # scenes shared by 64 scans
    scene = _Scene(np.random.default_rng(1000003 + scene_id), ground_ramp)
    elev, W = beam_layout(lidar)
    H = elev.shape[0]
    res_x = 2.0 * np.pi / W
    t_idx = np.arange(W, dtype=np.float64)
    phi = (W / 2 - t_idx) * res_x  # clockwise from the rear; atan2(x, y) = pi/2 + m res_x
    e = np.deg2rad(elev)
    ce, se = np.cos(e), np.sin(e)
    d = np.empty((W, H, 3))
    d[:, :, 0] = np.cos(phi)[:, None] * ce[None, :]
    d[:, :, 1] = np.sin(phi)[:, None] * ce[None, :]
    d[:, :, 2] = se[None, :]
    d = d.reshape(-1, 3)
    origin = np.array([0.5 * (seed % 64), rng.uniform(-0.5, 0.5), 0.0])
    if origin_xy is not None:
        origin[:2] = origin_xy
    if motion:
        dz, roll, pitch, yaw = sensor_attitude(seed)
        origin[2] += dz
        t = scene.cast(origin, d @ _rot_zyx(roll, pitch, yaw).T, max_range)
    else:
        t = scene.cast(origin, d, max_range)
    r = t + rng.normal(0.0, noise, size=t.shape)
    drop = rng.random(t.shape) < dropout
    r[drop | ~np.isfinite(t)] = np.nan
    pts = np.empty((d.shape[0], 4), dtype=np.float32)
    pts[:, :3] = (d * r[:, None]).astype(np.float32)
    pts[:, 3] = rng.integers(0, 101, size=t.shape).astype(np.float32)
    return pts


def make_symmetric_scan(seed: int, lidar: str = VLP16, quadrants: int = 4) -> np.ndarray:
    """A scan whose first quarter of azimuth columns is repeated, rotated by 90 degrees about the
    sensor, in the other quarters (quadrants = 4) or half repeated at 180 degrees (quadrants = 2).
    The rotations only swap and negate x / y, so every curvature (FA:817-848) repeats EXACTLY in
    each copy: the per-ring sort (FA:1172) meets ties everywhere and libstdc++'s order of equal
    values decides the order of the feature lists."""
    pts = make_scan(seed, lidar)
    _, W = beam_layout(lidar)
    H = pts.shape[0] // W
    step = W // quadrants
    base = pts[: step * H].copy()
    out = [base]
    cur = base
    for _ in range(quadrants - 1):
        nxt = cur.copy()
        if quadrants == 4:   # azimuth(t + W/4) = azimuth(t) - 90 deg: (x, y) -> (y, -x)
            nxt[:, 0], nxt[:, 1] = cur[:, 1], -cur[:, 0]
        else:                # 180 deg: (x, y) -> (-x, -y)
            nxt[:, 0], nxt[:, 1] = -cur[:, 0], -cur[:, 1]
        out.append(nxt)
        cur = nxt
    return np.concatenate(out, axis=0)


def make_batch(n_scans: int, lidar: str = VLP16, distinct: int | None = None, seed0: int = 1,
               motion: bool = False):
    """B raw scans packed as (float32 [sum N, 4], int64 offsets [B+1]).

    `distinct` scans are ray-cast (seeds seed0..) and tiled to fill the batch — the device work
    per scan is identical whether or not two slots carry the same cloud.
    """
    distinct = n_scans if distinct is None else max(1, min(distinct, n_scans))
    base = [make_scan(seed0 + k, lidar, motion=motion) for k in range(distinct)]
    scans = [base[k % distinct] for k in range(n_scans)]
    offsets = np.zeros(n_scans + 1, dtype=np.int64)
    offsets[1:] = np.cumsum([s.shape[0] for s in scans])
    return np.concatenate(scans, axis=0), offsets


def make_keyframes(n: int, seed: int = 7, corner: int = 400, surf: int = 1600, outlier: int = 250):
    """Synthetic MapOptimization keyframes: PointTypePose (x, y, z, roll, pitch, yaw) along a path
    that runs out ~90 m and back with uneven spacing (several poses share a 1 m key-pose voxel on the
    slow stretches, so the VoxelGrid of key poses averages indices), and per-keyframe corner / surf /
    outlier clouds in the keyframe's own frame (structure-like: points on a few planes and poles, so
    the 0.2 / 0.4 m VoxelGrids merge points within and across keyframes)."""
    rng = np.random.default_rng(seed)
    step = np.where(rng.random(n) < 0.3, 0.35, 2.8).astype(np.float32)
    half = n // 2
    s = np.concatenate([np.cumsum(step[:half]), np.cumsum(step[:half])[::-1][: n - half] - 0.7])
    poses = np.zeros((n, 6), np.float32)
    poses[:, 0] = s                                   # x (LOAM frame)
    poses[:, 1] = 0.05 * np.sin(s / 7.0)               # y
    poses[:, 2] = 3.0 * np.sin(s / 23.0)               # z
    poses[:, 3] = 0.01 * np.sin(s / 5.0)               # roll
    poses[:, 4] = 0.2 * np.sin(s / 31.0)               # pitch (heading in the camera-style frame)
    poses[:, 5] = 0.02 * np.cos(s / 11.0)              # yaw
    frames = []
    for k in range(n):
        def cloud(m, kind):
            pts = np.empty((m, 4), np.float32)
            u = rng.random((m, 3)).astype(np.float32)
            if kind == "pole":                        # vertical poles at fixed world-ish spots
                cx = np.floor(u[:, 0] * 8) * 5.0 - 20.0
                pts[:, 0] = cx + 0.05 * u[:, 1]
                pts[:, 1] = u[:, 2] * 4.0 - 1.5
                pts[:, 2] = np.floor(u[:, 1] * 6) * 4.0 - 12.0
            elif kind == "plane":                     # ground + walls
                w = np.floor(u[:, 0] * 3)
                pts[:, 0] = np.where(w == 0, u[:, 1] * 60 - 30, np.where(w == 1, -10.0, 12.0))
                pts[:, 1] = np.where(w == 0, -1.6, u[:, 2] * 5 - 1.6)
                pts[:, 2] = np.where(w == 0, u[:, 2] * 60 - 30, u[:, 1] * 60 - 30)
            else:                                     # scattered
                pts[:, :3] = (u - 0.5) * np.array([80, 20, 80], np.float32)
            pts[:, :3] += rng.normal(0, 0.02, (m, 3)).astype(np.float32)
            pts[:, 3] = (np.floor(rng.random(m) * 16) + np.floor(rng.random(m) * 1800) / 1e4).astype(np.float32)
            return pts
        frames.append((poses[k].copy(), cloud(corner, "pole"), cloud(surf, "plane"), cloud(outlier, "scatter")))
    return frames
