"""GPU parity of the projection on points placed at the row / column decision boundaries.

projectPointCloud (IP:305-336) truncates the float row quotient and rounds the double column
quotient. The device evaluates both with a multiply by the reciprocal and falls back to the
reference's division only when the quotient sits within a tolerance of an integer (row) or a
half-integer (column) — this test puts thousands of points within a few ulp of those boundaries
(and exactly on them, as far as float coordinates allow) and requires the cell of every point,
the range image and the cell -> point map to be bit-identical to the oracle's exact divisions.
"""
import numpy as np
import pytest

import oracle_py
from _compare import compare
from llsr import Pipeline, default_config

pytestmark = pytest.mark.gpu


def _boundary_points(cfg, n, seed):
    rng = np.random.default_rng(seed)
    H, W = cfg.num_vertical_scans, cfg.num_horizontal_scans
    res_x = np.float32(2 * np.pi / W)
    res_y = np.float32(np.deg2rad(cfg.vertical_angle_top - cfg.vertical_angle_bottom) / np.float32(H - 1))
    ang_b = np.float32(-(cfg.vertical_angle_bottom - 0.1) * np.pi / 180)
    r = rng.integers(0, H, n).astype(np.float64)
    k = rng.integers(0, W, n).astype(np.float64)
    # quotient offsets: exactly on, or a few ulp / tiny fractions around the boundaries
    dr = rng.choice([0.0, 1e-7, -1e-7, 3e-7, -3e-7, 1e-5, -1e-5, 0.5], n)
    dc = 0.5 + rng.choice([0.0, 1e-13, -1e-13, 1e-9, -1e-9, 1e-6, -1e-6, 0.25], n)
    va = (r + dr) * float(res_y) - float(ang_b)
    ha = np.pi / 2 + (k + dc) * float(res_x)
    R = rng.uniform(2.0, 60.0, n)
    z = R * np.sin(va)
    h = R * np.cos(va)
    pts = np.empty((n, 4), np.float32)
    pts[:, 0] = h * np.sin(ha)   # atan2(x, y) = ha
    pts[:, 1] = h * np.cos(ha)
    pts[:, 2] = z
    pts[:, 3] = rng.integers(0, 100, n)
    return pts


@pytest.mark.parametrize("lidar", ["vlp16", "hdl64e"])
def test_projection_boundaries_bit_exact(lidar, require_gpu):
    cfg = default_config(lidar, 1024 if lidar == "hdl64e" else None)
    pts = _boundary_points(cfg, 20000, 5 if lidar == "vlp16" else 6)
    pipe = Pipeline(cfg, max_batch=1, max_points=len(pts))
    g = pipe.process_scan(pts)
    o = oracle_py.Oracle(cfg).process(pts)
    assert np.array_equal(g["cell_point"], o["cell_point"])
    assert np.array_equal(g["range_image"].view(np.uint32), o["range_image"].view(np.uint32))
    assert not compare(g, o)
    pipe.close()
