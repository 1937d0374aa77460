"""CPU tests of the input wire formats (lego-loam-sr_amd/csrc/llsr_input.hip):
the KITTI .bin reader (host code of the C-ABI, runs without a GPU) against the reference loader's
restatement (oracle_py.kitti_read: IP:224-248, imageProjection.h:127-200), including its
1,000,000-float cap and partial trailing records, and argument validation of the PointCloud2
decoder (the decode itself runs on the device: tests/test_gpu_input.py)."""
import ctypes as C
import os

import numpy as np

import llsr
import oracle_py
from llsr import _abi


def _write(path, arr):
    np.asarray(arr, np.float32).tofile(path)


def test_kitti_count_and_read(tmp_path):
    d = tmp_path / "velodyne"
    d.mkdir()
    rng = np.random.default_rng(1)
    frames = [rng.normal(0, 20, (n, 4)).astype(np.float32) for n in (1000, 0, 3)]
    for k, f in enumerate(frames):
        _write(d / f"{k:06d}.bin", f)
    _write(d / "000005.bin", frames[0])            # gap: counting stops at the first missing index
    assert llsr.kitti_count(str(d)) == 3
    for k, f in enumerate(frames):
        got = llsr.kitti_read(str(d / f"{k:06d}.bin"))
        assert np.array_equal(got, f)
        assert np.array_equal(got, oracle_py.kitti_read(str(d / f"{k:06d}.bin")))


def test_kitti_read_caps_and_partial_records(tmp_path):
    big = np.arange(1000006, dtype=np.float32)      # 1e6 + 6 floats: the reference reads 1e6
    p = tmp_path / "big.bin"
    _write(p, big)
    got = llsr.kitti_read(str(p))
    assert got.shape == (250000, 4) and np.array_equal(got.reshape(-1), big[:1000000])
    assert np.array_equal(got, oracle_py.kitti_read(str(p)))
    q = tmp_path / "odd.bin"
    _write(q, np.arange(7, dtype=np.float32))      # 7 floats -> 1 point
    assert np.array_equal(llsr.kitti_read(str(q)), oracle_py.kitti_read(str(q)))
    assert llsr.kitti_read(str(q)).shape == (1, 4)


def test_kitti_read_missing_file(tmp_path):
    n = C.c_int32()
    assert llsr.lib().llsr_kitti_read(str(tmp_path / "none.bin").encode(), None, 0, C.byref(n)) == -5


def test_pc2_decode_rejects_bad_layouts():
    L = llsr.lib()
    msg = (_abi.Pc2Msg * 1)()
    msg[0].width, msg[0].height, msg[0].row_step = 4, 1, 64
    off = np.zeros(2, np.int64)
    bad_offset = llsr.pc2_layout([("x", 14, 7, 1)], 16)          # field runs past point_step
    assert L.llsr_decode_pointcloud2(C.byref(bad_offset), None, msg, 1, None, off.ctypes.data, None, None) == -22
    zero_step = llsr.pc2_layout([("x", 0, 7, 1)], 0)
    assert L.llsr_decode_pointcloud2(C.byref(zero_step), None, msg, 1, None, off.ctypes.data, None, None) == -22
    msg[0].height, msg[0].row_step = 2, 8                        # organized rows shorter than width*step
    ok = llsr.pc2_layout([("x", 0, 7, 1)], 16)
    assert L.llsr_decode_pointcloud2(C.byref(ok), None, msg, 1, None, off.ctypes.data, None, None) == -22


def test_pc2_restatement_field_matching():
    """The restatement maps only FLOAT32 / count-1 fields by name; others read 0."""
    n = 5
    rec = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("i16", "<u2"), ("pad", "u1", 2)])
    rec["x"], rec["y"], rec["z"], rec["i16"] = np.arange(n), 2 * np.arange(n), -np.arange(n), 7
    fields = [("x", 0, 7, 1), ("y", 4, 7, 1), ("z", 8, 7, 1), ("intensity", 12, 4, 1)]  # UINT16 intensity
    got = oracle_py.decode_pointcloud2(fields, 16, rec.tobytes(), n, 1, 16 * n)
    assert np.array_equal(got[:, 0], rec["x"]) and np.array_equal(got[:, 2], rec["z"])
    assert not got[:, 3].any()
