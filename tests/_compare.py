"""Field-by-field comparison of an llsr_scan_out result against the oracle's.

Bar: bit-exact for every array — integer / index / label arrays and every float
array, the VoxelGrid centroids of the less-flat cloud included: the device sums each voxel's points
in the order libstdc++'s std::sort leaves PCL's index_vector (llsr_fa.hip, exact_introsort with the
voxel-id comparator), as the oracle's PCL statement does.
"""
import numpy as np

from llsr import _abi


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
        r = diff_report(name, g, o)
        if r:
            errs.append(r)
    return errs
