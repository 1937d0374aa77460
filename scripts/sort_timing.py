"""Diagnostics: device time of the exact introsort (llsr_isort.h block_introsort, one 256-thread
workgroup) on the voxel ids of real less-flat rings and on synthetic inputs.

    python scripts/sort_timing.py [seed:ring ...]   (default: seed 5, rings 0, 3, .., 15)
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-sr_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import llsr  # noqa: E402
import oracle_py  # noqa: E402
from llsr import _abi, synth  # noqa: E402

f = llsr.lib().llsr_debug_exact_sort_ms
f.restype, f.argtypes = C.c_float, [C.c_void_p, C.c_int32, C.c_int32]


g = llsr.lib().llsr_debug_exact_sort_phases
g.restype, g.argtypes = C.c_int32, [C.c_void_p, C.c_int32, C.c_void_p]


def phases(a):
    """core clocks of one sort"""
    a = np.ascontiguousarray(a, np.float32)
    c = np.zeros(21, np.int64)
    assert g(a.ctypes.data, len(a), c.ctypes.data) == 0
    w = c[2:18].reshape(4, 4)
    return {"total": int(c[0]), "block": int(c[1]), "wave_partition": w[:, 0].tolist(), "small": w[:, 1].tolist(),
            "heap": w[:, 2].tolist(), "idle_end": w[:, 3].tolist()}


def t(a):
    a = np.ascontiguousarray(a, np.float32)
    return round(float(f(a.ctypes.data, len(a), 20)) * 1e3, 1)  # us


cfg = _abi.config_for("vlp16")
todo = [tuple(int(x) for x in a.split(":")) for a in sys.argv[1:]] or [(5, ring) for ring in range(0, 16, 3)]
scans = {}
res = {}
for seed, ring in todo:
    if seed not in scans:  # the first scan of a fresh pipeline, as the bench's distinct clouds
        scans[seed] = oracle_py.Oracle(cfg).process(synth.make_scan(seed, "vlp16"))
    r = scans[seed]
    loam, sr, er, lab = r["loam_xyzi"], r["start_ring_index"], r["end_ring_index"], r["label"]
    idx = np.arange(sr[ring], er[ring] + 1)
    p = loam[idx[lab[idx] <= 0]]
    inv = np.float32(5.0)
    mn = p[:, :3].min(0)
    mx = p[:, :3].max(0)
    minb = np.floor(mn * inv).astype(np.int64)
    div = np.floor(mx * inv).astype(np.int64) - minb + 1
    i = (np.floor(p[:, :3] * inv) - minb.astype(np.float32)).astype(np.int64)
    v = (i[:, 0] + i[:, 1] * div[0] + i[:, 2] * div[0] * div[1]).astype(np.float32)
    n = len(v)
    rng = np.random.default_rng(ring)
    res[f"seed{seed}_ring{ring}"] = {"n": n, "voxel_ids_us": t(v), "voxel_ids_phase_clocks": phases(v),
                                      "all_equal_phase_clocks": phases(np.zeros(n)), "random_us": t(rng.random(n)), "sorted_us": t(np.arange(n)),
                          "few_values_us": t(rng.integers(0, 8, n)), "all_equal_us": t(np.zeros(n))}
print(json.dumps(res))
