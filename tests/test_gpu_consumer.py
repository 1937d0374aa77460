"""The drop-in boundary from a compiled C++ caller: tests/native/consumer.cpp,
built against include/llsr.h and linked with libllsr.so, makes the calls the ROS nodes make, in
its own process:

* ipfa: repacks PCL-layout points and calls llsr_process_scan for three consecutive VLP-16 scans
  (FA carry-over state included); outputs equal, bit for bit, the oracle (tests/_compare.py) and
  the same calls made through the ctypes binding;
* s2s: llsr_scan2scan over a drive's consecutive problems with the node's transformCur /
  isDegenerate carried between calls, against oracle_py.scan2scan (FA:2505-2535);
* s2m: llsr_scan2map on the map fixture's problems against oracle_py.scan2map (MO:1572-1610);
* mapping: llsr_mapping_init / _batch / _fetch / _keyposes over a VLP-16 drive uploaded to HBM
  with hipMemcpy, against oracle_py.OracleMapping (MO:1854-1896).
Bar: bit-exact everywhere."""
import ctypes
import os
import struct
import subprocess

import numpy as np
import pytest

import oracle_py
from llsr import Pipeline, _abi, default_config, synth

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "tests", "native", "llsr_consumer")


def _read_out(path, n_scans):
    raw = open(path, "rb").read()
    pos = 0

    def take(dt, n):
        nonlocal pos
        a = np.frombuffer(raw, dt, n, pos)
        pos += a.nbytes
        return a

    res = []
    for _ in range(n_scans):
        n_points, S, O, M, Ms, F, L, H = take(np.int32, 8)
        r = dict(n_points=n_points, n_segmented=S, n_outlier=O, n_less_sharp=M, n_sharp=Ms, n_flat=F, n_less_flat=L)
        r["orientation"] = take(np.float32, 3)
        r["start_ring_index"] = take(np.int32, H)
        r["end_ring_index"] = take(np.int32, H)
        r["seg_xyzi"] = take(np.float32, 4 * S).reshape(-1, 4)
        r["seg_ground_flag"] = take(np.uint8, S)
        r["seg_col_ind"] = take(np.uint32, S)
        r["seg_range"] = take(np.float32, S)
        r["outlier_xyzi"] = take(np.float32, 4 * O).reshape(-1, 4)
        r["loam_xyzi"] = take(np.float32, 4 * S).reshape(-1, 4)
        r["less_sharp_ind"] = take(np.int32, M)
        r["sharp_ind"] = take(np.int32, Ms)
        r["flat_ind"] = take(np.int32, F)
        r["less_flat_xyzi"] = take(np.float32, 4 * L).reshape(-1, 4)
        res.append(r)
    assert pos == len(raw)
    return res


def test_cxx_consumer_matches_ctypes(require_gpu, tmp_path):
    assert os.path.exists(EXE), "tests/native/llsr_consumer is built by __graft_entry__.build()"
    scans = [synth.make_scan(s, "vlp16") for s in (31, 32, 33)]
    inp, out = tmp_path / "scans.bin", tmp_path / "out.bin"
    with open(inp, "wb") as f:
        f.write(np.int32(len(scans)).tobytes())
        for sc in scans:
            f.write(np.int32(len(sc)).tobytes())
            f.write(np.ascontiguousarray(sc, np.float32).tobytes())
    r = subprocess.run([EXE, "ipfa", str(inp), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = _read_out(out, len(scans))
    pipe = Pipeline(default_config("vlp16"), device=0, max_batch=1, max_points=40000)
    ora = oracle_py.Oracle(default_config("vlp16"))
    errs = []
    for k, sc in enumerate(scans):
        ref = pipe.process_scan(sc)
        o = ora.process(sc)
        for key, v in got[k].items():
            if not np.array_equal(np.asarray(v), np.asarray(ref[key])):
                errs.append(f"scan {k}: {key} differs from the ctypes path")
            if key in o and not np.array_equal(np.asarray(v), np.asarray(o[key])):
                errs.append(f"scan {k}: {key} differs from the oracle")
    pipe.close()
    assert not errs, "\n".join(errs)


def _f4(a):
    return np.ascontiguousarray(a, np.float32).reshape(-1, 4)


def _run(mode, payload: bytes, tmp_path, timeout=120):
    inp, out = tmp_path / f"{mode}.in", tmp_path / f"{mode}.out"
    inp.write_bytes(payload)
    r = subprocess.run([EXE, mode, str(inp), str(out)], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr
    return out.read_bytes()


def test_cxx_consumer_scan2scan(require_gpu, tmp_path):
    cfg = default_config("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    od = oracle_py.OracleOdometry(cfg)
    probs = []
    prev = None
    for k in range(4):  # consecutive scans of one drive: the LM inputs of frames 2..4
        r = od.ora.process(synth.make_scan(41 + k, "vlp16"))
        loam = r["loam_xyzi"]
        cur = {"sharp": loam[r["sharp_ind"]], "flat": np.concatenate([loam[r["flat_ind"]], od.shadow]),
               "less_sharp": loam[r["less_sharp_ind"]], "less_flat": r["less_flat_xyzi"]}
        if prev is not None:
            probs.append((cur["sharp"], cur["flat"], prev["less_sharp"],
                          np.concatenate([prev["less_flat"], od.shadow])))
        prev = cur
    t0 = np.zeros(6, np.float32)
    payload = struct.pack("<i", len(probs)) + t0.tobytes() + struct.pack("<i", 0)
    for pr in probs:
        payload += struct.pack("<4i", *(len(c) for c in pr)) + b"".join(_f4(c).tobytes() for c in pr)
    raw = _run("s2s", payload, tmp_path)
    n = ctypes.sizeof(_abi.S2SReport)
    tcur, deg = t0.copy(), 0
    pos = 0
    for p, pr in enumerate(probs):
        g_t = np.frombuffer(raw, np.float32, 6, pos)
        g_deg = struct.unpack_from("<i", raw, pos + 24)[0]
        g_rep = _abi.S2SReport.from_buffer_copy(raw[pos + 28:pos + 28 + n]).as_dict()
        pos += 28 + n
        o = oracle_py.scan2scan(cfg, *pr, tcur, deg)
        tcur, deg = o["transform_cur"], o["is_degenerate"]
        assert np.array_equal(g_t, tcur), (p, g_t, tcur)
        assert g_deg == deg
        for key in ("surf_iterations", "corner_iterations", "n_surf_corr", "n_corner_corr", "skipped"):
            assert g_rep[key] == o[key], (p, key, g_rep[key], o[key])
    assert pos == len(raw)


def test_cxx_consumer_scan2map(require_gpu, tmp_path):
    z = np.load(os.path.join(REPO, "tests", "golden", "mo_map_vlp16.npz"))
    cfg = default_config("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    probs = [(z[f"q{i}_corner"], z[f"q{i}_surf"], z["corner_map"], z["surf_map"], z[f"q{i}_init"])
             for i in range(int(z["n_queries"]))]
    payload = struct.pack("<i", len(probs))
    for pr in probs:
        payload += struct.pack("<4i", *(len(c) for c in pr[:4])) + b"".join(_f4(c).tobytes() for c in pr[:4])
        payload += np.ascontiguousarray(pr[4], np.float32).tobytes()
    raw = _run("s2m", payload, tmp_path)
    n = ctypes.sizeof(_abi.LmReport)
    pos = 0
    for p, pr in enumerate(probs):
        g_pose = np.frombuffer(raw, np.float32, 6, pos)
        g = _abi.LmReport.from_buffer_copy(raw[pos + 24:pos + 24 + n]).as_dict()
        pos += 24 + n
        o = oracle_py.scan2map(cfg, *pr)
        assert np.array_equal(g_pose, o["pose"]), (p, g_pose, o["pose"])
        for key in ("iterations", "converged", "degenerate", "n_corner_corr", "n_surf_corr", "min_lambda", "cf_mean"):
            assert np.array_equal(np.asarray(g[key]), np.asarray(o[key])), (p, key, g[key], o[key])
    assert pos == len(raw)


def test_cxx_consumer_mapping_chain(require_gpu, tmp_path):
    cfg = default_config("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    scans = [synth.make_scan(150 + k, "vlp16") for k in range(4)]
    payload = struct.pack("<ii", _abi.LLSR_MODE_LM_APPLIED, len(scans))
    for sc in scans:
        payload += struct.pack("<i", len(sc)) + _f4(sc).tobytes()
    raw = _run("mapping", payload, tmp_path)
    n = ctypes.sizeof(_abi.MappingSlot)
    om = oracle_py.OracleMapping(cfg, _abi.LLSR_MODE_LM_APPLIED)
    pos = 0
    for k, sc in enumerate(scans):
        g = _abi.MappingSlot.from_buffer_copy(raw[pos:pos + n])
        pos += n
        o = om.process(sc)
        assert g.frames == o["frames"]
        if not o["step"]:
            continue
        assert g.keyframes == o["keyframes"] and bool(g.lm_ran) == bool(o["lm_ran"])
        for key in ("transform_sum", "transform_tobe_mapped", "transform_bef_mapped", "transform_aft_mapped"):
            assert np.array_equal(np.array(getattr(g, key)[:], np.float32), o[key]), (k, key)
    K = struct.unpack_from("<i", raw, pos)[0]
    kp = np.frombuffer(raw, np.float32, 6 * K, pos + 4).reshape(K, 6)
    assert np.array_equal(kp, np.array(om.keyposes, np.float32).reshape(-1, 6))
