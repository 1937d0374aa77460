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


def _clouds(b, pos, n):
    out = []
    for _ in range(n):
        k = int(np.frombuffer(b, np.int32, 1, pos)[0])
        pos += 4
        out.append(np.frombuffer(b, np.float32, 4 * k, pos).reshape(k, 4))
        pos += 16 * k
    return out, pos


def _read_drive(path):
    b = open(path, "rb").read()
    pos = 0
    nf = int(np.frombuffer(b, np.int32, 1, pos)[0])
    pos += 4
    fa = []
    for _ in range(nf):
        hdr = np.frombuffer(b, np.int32, 9, pos)
        pos += 36
        t = np.frombuffer(b, np.float32, 12, pos)
        pos += 48
        cl, pos = _clouds(b, pos, 8)
        keys = ("sharp", "less_sharp", "flat", "less_flat", "corner_last", "surf_last", "corner_scan", "surf_scan")
        r = dict(zip(keys, cl))
        r.update(seq=int(hdr[0]), lm=int(hdr[1]), is_degenerate=int(hdr[2]), surf_iterations=int(hdr[3]),
                 corner_iterations=int(hdr[4]), n_surf_corr=int(hdr[5]), n_corner_corr=int(hdr[6]),
                 degenerate=int(hdr[7]), skipped=int(hdr[8]), transform_cur=t[:6], transform_sum=t[6:])
        fa.append(r)
    nm = int(np.frombuffer(b, np.int32, 1, pos)[0])
    pos += 4
    mo = []
    for _ in range(nm):
        seq = int(np.frombuffer(b, np.int32, 1, pos)[0])
        pose = np.frombuffer(b, np.float32, 6, pos + 4)
        its = int(np.frombuffer(b, np.int32, 1, pos + 28)[0])
        pos += 32
        mo.append({"seq": seq, "pose": pose, "iterations": its})
    assert pos == len(b)
    return fa, mo


def _bits_equal(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("lidar,frames,seed0", [("vlp16", 6, 40), ("hdl64e", 3, 5)])
def test_adapter_threads_drive_matches_oracle(require_gpu, tmp_path, lidar, frames, seed0):
    """The reference's thread layout (main.cpp:10-11, channel.h:24-54, FA:2742-2853) through the
    adapter: IP thread (Projection::run + handoff into ProjectionOut, blocking send), FA thread
    (Odometry::step on its own handle: update_transformation, integrateTransformation,
    publishCloudsLast), MO thread (scan2map_optimization on a third handle, non-blocking send).
    A 6-frame moving VLP-16 drive (and a 3-frame HDL-64E one): every frame's feature clouds, LM report, transformCur /
    transformSum and last / scan clouds bit-exact against oracle_py.OracleOdometry, and every
    scan-to-map problem MO received bit-exact against oracle_py.scan2map (map: the drive's first
    last clouds, pose 0)."""
    import oracle_py
    from llsr import _abi, default_config, synth
    assert os.path.exists(NODE), "build with make -C lego-loam-sr_amd"
    cfg = default_config(lidar)
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    F = frames
    frames = [np.ascontiguousarray(synth.make_scan(seed0 + k, lidar, motion=True), np.float32) for k in range(F)]
    ora = oracle_py.OracleOdometry(cfg)
    outs = [ora.process(p) for p in frames]
    corner_map, surf_map = outs[0]["corner_last"], outs[0]["surf_last"]
    fpath, mpath, opath = tmp_path / "frames.bin", tmp_path / "map.bin", tmp_path / "out.bin"
    with open(fpath, "wb") as f:
        np.int32(F).tofile(f)
        for p in frames:
            np.int32(len(p)).tofile(f)
            p.tofile(f)
    with open(mpath, "wb") as f:
        for c in (corner_map, surf_map):
            np.int32(len(c)).tofile(f)
            np.ascontiguousarray(c, np.float32).tofile(f)
        np.zeros(6, np.float32).tofile(f)
    code = {"vlp16": _abi.LLSR_LIDAR_VLP16, "hdl64e": _abi.LLSR_LIDAR_HDL64E}[lidar]
    r = subprocess.run([NODE, "drive", str(code), str(fpath), str(mpath), str(opath)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    fa, mo = _read_drive(opath)
    assert [x["seq"] for x in fa] == list(range(F))
    errs, surf_its = [], []
    for k, (g, o) in enumerate(zip(fa, outs)):
        feat = o["features"]
        loam = feat["loam_xyzi"][: feat["n_segmented"]]
        from llsr import shadow_points
        want = {"sharp": loam[feat["sharp_ind"]], "less_sharp": loam[feat["less_sharp_ind"]],
                "flat": np.concatenate([loam[feat["flat_ind"]], shadow_points()]),
                "less_flat": feat["less_flat_xyzi"]}
        for key, ref in want.items():
            if not _bits_equal(g[key], ref):
                errs.append(f"frame {k}: {key} differs")
        if g["lm"] != (o["lm"] is not None):
            errs.append(f"frame {k}: lm ran {g['lm']} vs oracle {o['lm'] is not None}")
        elif o["lm"] is not None:
            surf_its.append(o["lm"]["surf_iterations"])
            for key in ("surf_iterations", "corner_iterations", "n_surf_corr", "n_corner_corr", "degenerate",
                        "skipped"):
                if g[key] != o["lm"][key]:
                    errs.append(f"frame {k}: lm {key} {g[key]} vs {o['lm'][key]}")
            if g["is_degenerate"] != int(o["lm"]["is_degenerate"]):
                errs.append(f"frame {k}: isDegenerate {g['is_degenerate']} vs {o['lm']['is_degenerate']}")
        for key in ("transform_cur", "transform_sum", "corner_last", "surf_last"):
            if not _bits_equal(g[key], o[key]):
                errs.append(f"frame {k}: {key} {g[key] if key.startswith('t') else g[key].shape} vs "
                            f"{o[key] if key.startswith('t') else o[key].shape}")
        for key in ("corner_scan", "surf_scan"):
            ref = o[key] if o[key] is not None else np.zeros((0, 4), np.float32)
            if not _bits_equal(g[key], ref):
                errs.append(f"frame {k}: {key} differs")
    assert max(surf_its) >= (2 if lidar == "vlp16" else 1), f"the drive never iterates the surf step: {surf_its}"
    assert mo, "MO received no AssociationOut"
    for m in mo:
        o = outs[m["seq"]]
        om = oracle_py.scan2map(cfg, o["corner_scan"], o["surf_scan"], corner_map, surf_map, np.zeros(6, np.float32))
        if not _bits_equal(m["pose"], om["pose"]) or m["iterations"] != om["iterations"]:
            errs.append(f"MO frame {m['seq']}: pose {m['pose']} / {m['iterations']} it vs {om['pose']} / "
                        f"{om['iterations']} it")
    assert not errs, "\n".join(errs)
