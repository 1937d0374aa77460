"""GPU parity of the projection on points placed at the row / column decision boundaries.

projectPointCloud (IP:305-336) truncates the float row quotient of asinf and rounds the double
column quotient of atan2f. The device decides both with a certified fast path (fdlibm's asinf
polynomial, a minimax atan2 and reciprocal multiplies; csrc/llsr_ip.hip project_cell_fast) and
falls back to the bit-exact libm ports and the reference's divisions only when a quotient sits
within the path's error bound of an integer (row) or a half-integer (column). These tests put
thousands of points within a few ulp of those boundaries (and exactly on them, as far as float
coordinates allow), and at uniformly random directions, and require the cell of every point, the
range image and the cell -> point map to be bit-identical to the oracle's exact libm projection.
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


@pytest.mark.parametrize("lidar", ["vlp16", "hdl64e"])
def test_projection_random_directions_bit_exact(lidar, require_gpu):
    """Uniformly random directions (no bin-centred angles): every point's cell from the certified
    fast path (or its exact fallback) equals the oracle's libm projection, incl. |z/r| >= 0.5,
    points on the axes (x or y == 0) and ranges below the 0.1 m cut."""
    cfg = default_config(lidar, 1024 if lidar == "hdl64e" else None)
    rng = np.random.default_rng(21 if lidar == "vlp16" else 22)
    n = 30000
    v = rng.normal(size=(n, 3))
    v[:, 2] *= 0.3
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    R = np.exp(rng.uniform(np.log(0.05), np.log(80.0), n))
    pts = np.zeros((n, 4), np.float32)
    pts[:, :3] = v * R[:, None]
    pts[:200, 0] = 0.0   # on the axes: the fast path defers these to the exact atan2f
    pts[200:400, 1] = 0.0
    pts[:, 3] = rng.integers(0, 100, n)
    pipe = Pipeline(cfg, max_batch=1, max_points=n)
    g = pipe.process_scan(pts)
    o = oracle_py.Oracle(cfg).process(pts)
    assert np.array_equal(g["cell_point"], o["cell_point"])
    assert np.array_equal(g["range_image"].view(np.uint32), o["range_image"].view(np.uint32))
    pipe.close()
