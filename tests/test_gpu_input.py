"""GPU parity of the input wire formats (llsr_input.hip):

* PointCloud2 -> PointXYZI (pcl::fromROSMsg, IP:196) on the device, bit-exact (NaN payloads
  included) against the numpy restatement oracle_py.decode_pointcloud2, for the velodyne_pointcloud
  layout (point_step 32), a packed unaligned layout (point_step 22), an organized cloud with row
  padding, and layouts whose intensity / x fields do not map (wrong datatype / absent);
* decode -> llsr_process_batch gives exactly the outputs of the float4 cloud itself;
* llsr_kitti_load (pinned upload of B frames) equals the reference loader's restatement.
"""
import numpy as np
import pytest

import llsr
import oracle_py
from _compare import compare
from llsr import Pipeline, default_config, synth

pytestmark = pytest.mark.gpu

VELODYNE = ([("x", 0, 7, 1), ("y", 4, 7, 1), ("z", 8, 7, 1), ("intensity", 16, 7, 1), ("ring", 20, 4, 1),
             ("time", 24, 7, 1)], 32)
PACKED = ([("x", 0, 7, 1), ("y", 4, 7, 1), ("z", 8, 7, 1), ("intensity", 12, 7, 1), ("ring", 16, 4, 1),
           ("time", 18, 7, 1)], 22)


def _encode(xyzi, fields, step, width=None, height=1, row_pad=0, rng=None):
    """Pack float4 points into a PointCloud2 byte buffer of the given layout (other fields random)."""
    rng = rng or np.random.default_rng(0)
    n = len(xyzi)
    width = width if width is not None else n
    row_step = width * step + row_pad
    buf = np.frombuffer(rng.bytes(max(row_step * height, 1)), np.uint8).copy()[:row_step * height]
    src = {"x": 0, "y": 1, "z": 2, "intensity": 3}
    k = np.arange(n)
    base = (k // max(width, 1)) * row_step + (k % max(width, 1)) * step
    for name, off, dt, cnt in fields:
        if name in src and dt == 7 and n:
            col = np.ascontiguousarray(xyzi[:, src[name]], np.float32).view(np.uint8).reshape(n, 4)
            buf[(base + off)[:, None] + np.arange(4)[None, :]] = col
    return buf.tobytes(), width, height, row_step


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _check(fields, step, msgs):
    lay = llsr.pc2_layout(fields, step)
    got, off, d_off = llsr.decode_pointcloud2(lay, msgs)
    g = got.cpu().numpy()
    for b, (data, w, h, rs) in enumerate(msgs):
        ref = oracle_py.decode_pointcloud2(fields, step, data, w, h, rs)
        assert np.array_equal(_bits(g[off[b]:off[b + 1]]), _bits(ref)), b
    assert np.array_equal(d_off.cpu().numpy(), off)
    return got, off, d_off


def test_decode_velodyne_and_packed_layouts(require_gpu):
    rng = np.random.default_rng(3)
    for fields, step in (VELODYNE, PACKED):
        msgs = []
        for n in (1200, 0, 1, 777):
            pts = rng.normal(0, 20, (n, 4)).astype(np.float32)
            if n > 10:
                pts[5:9, :3] = np.nan                      # removeNaNFromPointCloud runs later
            msgs.append(_encode(pts, fields, step, rng=rng))
        _check(fields, step, msgs)


def test_decode_organized_and_unmapped_fields(require_gpu):
    rng = np.random.default_rng(4)
    pts = rng.normal(0, 5, (16 * 90, 4)).astype(np.float32)
    msg = _encode(pts, VELODYNE[0], 32, width=90, height=16, row_pad=12, rng=rng)
    _check(VELODYNE[0], 32, [msg])
    # intensity as UINT16 and x as FLOAT64: PCL does not map them (they read 0)
    odd = [("x", 0, 8, 1), ("y", 8, 7, 1), ("z", 12, 7, 1), ("intensity", 16, 4, 1)]
    _check(odd, 20, [(rng.bytes(20 * 50), 50, 1, 1000)])


def test_decode_then_process_matches_direct(require_gpu):
    import torch
    cfg = default_config("vlp16")
    scans = [synth.make_scan(s) for s in (3, 4, 5)]
    msgs = [_encode(s, *VELODYNE) for s in scans]
    got, off, d_off = _check(*VELODYNE, msgs)
    pa = Pipeline(cfg, max_batch=3, max_points=max(len(s) for s in scans))
    pb = Pipeline(cfg, max_batch=3, max_points=max(len(s) for s in scans))
    d_pts = torch.from_numpy(np.concatenate(scans)).cuda()
    torch.cuda.synchronize()
    pa.process_batch(got.data_ptr(), d_off.data_ptr(), 3)
    pb.process_batch(d_pts.data_ptr(), d_off.data_ptr(), 3)
    for b in range(3):
        assert not compare(pa.fetch(b), pb.fetch(b)), b
    pa.close()
    pb.close()


def test_kitti_load(tmp_path, require_gpu):
    d = tmp_path / "velodyne"
    d.mkdir()
    rng = np.random.default_rng(8)
    frames = [rng.normal(0, 30, (n, 4)).astype(np.float32) for n in (5000, 1, 0, 12345)]
    for k, f in enumerate(frames):
        f.tofile(d / f"{k:06d}.bin")
    pts, off, d_off = llsr.kitti_load(str(d), 0, 4, cap_points=20000)
    p = pts.cpu().numpy()
    for k in range(4):
        assert np.array_equal(_bits(p[off[k]:off[k + 1]]), _bits(oracle_py.kitti_read(str(d / f"{k:06d}.bin"))))
    assert np.array_equal(d_off.cpu().numpy(), off)
