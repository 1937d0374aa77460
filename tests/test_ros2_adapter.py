"""The ROS2 node-side adapter (integration/ros2/llsr_ros2.hpp), the code the reference's nodes call
in place of their per-scan arithmetic (imageProjection.cpp:189-222, featureAssociation.cpp:2769-2775
and 1310-1314, 2505-2535; mapOptmization.cpp:1572-1610). No ROS in this image: the adapter is
templated on the message / cloud types and tests/native/ros2_adapter_check.cpp instantiates it with
plain structs carrying the field names of cloud_msgs/CloudInfo, ProjectionOut and
pcl::PointCloud<PointXYZI>.

* CPU: the marshalling (llsr_scan_out -> CloudInfo / ProjectionOut / feature clouds) on a hand-made
  scan output, every field checked.
* GPU: the adapter's Projection class on one synthetic scan, its CloudInfo arrays and clouds
  compared bit for bit with the ctypes pipeline's outputs and the oracle's.
"""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "native", "ros2_adapter_check.cpp")
NODE = os.path.join(REPO, "tests", "native", "llsr_ros2_node")


def test_adapter_marshalling(tmp_path):
    exe = str(tmp_path / "ros2_adapter_check")
    subprocess.run(["g++", "-O1", "-std=c++11", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(REPO, "include"),
                    "-o", exe, SRC], check=True)
    r = subprocess.run([exe, "marshal"], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr


def _read(path):
    b = open(path, "rb").read()
    pos = 0

    def take(dtype, n):
        nonlocal pos
        a = np.frombuffer(b, dtype, n, pos)
        pos += a.nbytes
        return a

    def cloud():
        n = int(take(np.int32, 1)[0])
        return take(np.float32, 4 * n).reshape(n, 4)

    H = int(take(np.int32, 1)[0])
    out = {"start": take(np.int32, H), "end": take(np.int32, H), "orientation": take(np.float32, 3)}
    S = int(take(np.int32, 1)[0])
    out.update(gflag=take(np.uint8, S), col=take(np.uint32, S), range=take(np.float32, S))
    for k in ("segmented", "outlier", "loam", "sharp", "less_sharp", "flat", "less_flat"):
        out[k] = cloud()
    assert pos == len(b)
    return out


@pytest.mark.gpu
def test_adapter_node_matches_pipeline(require_gpu, tmp_path):
    import oracle_py
    from llsr import Pipeline, _abi, default_config, shadow_points, synth
    assert os.path.exists(NODE), "build with make -C lego-loam-sr_amd"
    cfg = default_config("vlp16")
    pts = np.ascontiguousarray(synth.make_scan(3, "vlp16"), np.float32)
    inp, outp = tmp_path / "in.bin", tmp_path / "out.bin"
    pts.tofile(inp)
    r = subprocess.run([NODE, "node", str(_abi.LLSR_LIDAR_VLP16), str(inp), str(outp)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    a = _read(outp)
    pipe = Pipeline(cfg, max_points=40000)
    g = pipe.process_scan(pts)
    pipe.close()
    o = oracle_py.Oracle(cfg).process(pts)
    for ref in (g, o):
        S = ref["n_segmented"]
        assert np.array_equal(a["start"], ref["start_ring_index"]) and np.array_equal(a["end"], ref["end_ring_index"])
        assert np.array_equal(a["orientation"].view(np.uint32), np.asarray(ref["orientation"], np.float32).view(np.uint32))
        assert np.array_equal(a["gflag"], ref["seg_ground_flag"][:S].astype(np.uint8))
        assert np.array_equal(a["col"], ref["seg_col_ind"][:S])
        assert np.array_equal(a["range"].view(np.uint32), ref["seg_range"][:S].view(np.uint32))
        assert np.array_equal(a["segmented"].view(np.uint32), ref["seg_xyzi"][:S].view(np.uint32))
        assert np.array_equal(a["outlier"].view(np.uint32), ref["outlier_xyzi"].view(np.uint32))
        loam = ref["loam_xyzi"][:S]
        assert np.array_equal(a["loam"].view(np.uint32), loam.view(np.uint32))
        assert np.array_equal(a["sharp"], loam[ref["sharp_ind"]])
        assert np.array_equal(a["less_sharp"], loam[ref["less_sharp_ind"]])
        flat = np.concatenate([loam[ref["flat_ind"]], shadow_points()])
        assert np.array_equal(a["flat"].view(np.uint32), flat.view(np.uint32))
        assert np.array_equal(a["less_flat"].view(np.uint32), ref["less_flat_xyzi"].view(np.uint32))
