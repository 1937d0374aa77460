"""Field-by-field comparison of an llsr_scan_out result against the oracle's.

Bar: bit-exact for every integer / index / label array and for every float array
that is a copy or a deterministic function of the input (range image, clouds, curvature,
orientation); VoxelGrid centroids (less-flat cloud) within max(1e-5, 1e-6 |x|) because PCL sums a
voxel's points in std::sort's tie order (the device sums them in input order).
"""
import numpy as np

from llsr import _abi

LESS_FLAT_ATOL = 1e-5  # absolute, for |value| <= 1
LESS_FLAT_RTOL = 1e-6  # relative beyond (intensity = ring + time reaches 64 on HDL-64E)


def _bits(a):
    a = np.asarray(a)
    if a.dtype == np.float32:
        return a.view(np.uint32)
    return a


def diff_report(name, g, o, limit=5):
    g, o = np.asarray(g), np.asarray(o)
    if g.shape != o.shape:
        return f"{name}: shape {g.shape} vs oracle {o.shape}"
    if g.size == 0:
        return None
    gb, ob = _bits(g), _bits(o)
    if gb.ndim > 1:
        gb, ob = gb.reshape(gb.shape[0], -1), ob.reshape(ob.shape[0], -1)
        bad = np.nonzero(np.any(gb != ob, axis=1))[0]
    else:
        bad = np.nonzero(gb != ob)[0]
    if bad.size == 0:
        return None
    rows = ", ".join(f"[{k}] gpu={g[k].tolist()} oracle={o[k].tolist()}" for k in bad[:limit])
    return f"{name}: {bad.size} mismatching entries, first: {rows}"


def compare(gpu: dict, ora: dict, skip=()):
    """Return a list of human-readable mismatch descriptions (empty = parity)."""
    errs = []
    for k in _abi.COUNTS:
        if gpu[k] != ora[k]:
            errs.append(f"{k}: gpu={gpu[k]} oracle={ora[k]}")
    r = diff_report("orientation", gpu["orientation"], ora["orientation"])
    if r:
        errs.append(r)
    for name, *_ in _abi.ARRAYS:
        if name in skip:
            continue
        g, o = gpu[name], ora[name]
        if name == "less_flat_xyzi":
            if g.shape != o.shape:
                errs.append(f"{name}: shape {g.shape} vs {o.shape}")
            elif g.size and not np.all(np.abs(g - o) <= np.maximum(LESS_FLAT_ATOL, LESS_FLAT_RTOL * np.abs(o))):
                k = int(np.argmax(np.abs(g - o).max(axis=1)))
                errs.append(f"{name}: max |d| {np.abs(g - o).max():.3g} at {k}: {g[k]} vs {o[k]}")
            continue
        r = diff_report(name, g, o)
        if r:
            errs.append(r)
    return errs
