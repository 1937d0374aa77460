"""The drop-in boundary from a compiled C++ caller: tests/native/consumer.cpp,
built against include/llsr.h and linked with libllsr.so, repacks PCL-layout points and calls
llsr_process_scan for three consecutive VLP-16 scans (FA carry-over state included) in its own
process; its outputs must equal, bit for bit, the same calls made through the ctypes binding."""
import os
import subprocess

import numpy as np
import pytest

from llsr import Pipeline, default_config, synth

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
    r = subprocess.run([EXE, str(inp), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = _read_out(out, len(scans))
    pipe = Pipeline(default_config("vlp16"), device=0, max_batch=1, max_points=40000)
    errs = []
    for k, sc in enumerate(scans):
        ref = pipe.process_scan(sc)
        for key, v in got[k].items():
            if not np.array_equal(np.asarray(v), np.asarray(ref[key])):
                errs.append(f"scan {k}: {key} differs")
    pipe.close()
    assert not errs, "\n".join(errs)
