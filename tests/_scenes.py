"""Scenes that drive the LMs into their degenerate branch (FA:1959-1990, MO:1507-1537).

The reference scans the eigenvalues from the LARGEST down and stops at the first one above the
threshold (10 in FA, 100 in MO), so the branch fires only when every eigenvalue of AtA is below
it: a handful of correspondences on points close to the sensor. Then every row of matV2 is zeroed,
matP = matV.inverse() * 0 and matX = matP * matX2 are (signed) zeros, the pose does not move and
the loop stops at iteration 0. These scenes shrink the synthetic street around the sensor (scale
f) and keep a few queries, which is how the degenerate branch is reached here."""
import os

import numpy as np

import oracle_py
from llsr import default_config, synth

# the one-lane 76k map (tests/golden/make_mo_fixture.py, mo_map_vlp16_small.npz)
FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mo_map_vlp16_small.npz")


def _scaled(a, f):
    b = np.array(a, np.float32, copy=True)
    b[:, :3] *= np.float32(f)
    return b


def fa_degenerate_pairs(n=6):
    """(cfg, [(sharp, flat, corner_last, surf_last, t0)]) whose corner phase is degenerate."""
    cfg = default_config("vlp16")
    ora = oracle_py.Oracle(cfg)
    prev = ora.process(synth.make_scan(1, "vlp16"))
    cur = ora.process(synth.make_scan(2, "vlp16"))
    sharp, flat, cl, sl = oracle_py.fa_lm_inputs(prev, cur)
    out = []
    for k in range(n):
        idx = (np.arange(10 + k % 3) * 7 + 3 * k) % len(sharp)
        t0 = np.array([0.0, 0.03, 0.0, 0.1, 0.0, 0.1], np.float32) * np.float32(k % 2)
        out.append((_scaled(sharp[idx], 0.1), _scaled(flat, 0.1), _scaled(cl, 0.1), _scaled(sl, 0.1), t0))
    return cfg, out


# flat-query offsets k of fa_degenerate_surf_pairs whose surf step is degenerate at iteration 0
# (every AtA eigenvalue below 10), and offsets with fewer than 10 surf correspondences (every surf
# iteration skipped); found by the oracle, re-checked by tests/test_degenerate.py
FA_DEGENERATE_SURF_CASES = (8, 10, 17)
FA_SURF_SKIP_CASES = (0, 4)


def fa_degenerate_surf_pairs():
    """(cfg, [(sharp, flat, corner_last, surf_last, t0, is_degenerate_in)]): frames 1 -> 2 of the
    moving drive shrunk 10x with 12 flat queries (offset k) and 5 sharp ones (the corner step
    never reaches 10 correspondences, so it skips every iteration and the flag it leaves is the
    surf step's), each with isDegenerate carried in as 0 and as 1."""
    cfg = default_config("vlp16")
    ora = oracle_py.Oracle(cfg)
    prev = ora.process(synth.make_scan(1, "vlp16", motion=True))
    cur = ora.process(synth.make_scan(2, "vlp16", motion=True))
    sharp, flat, cl, sl = oracle_py.fa_lm_inputs(prev, cur)
    n = len(flat) - 160  # the scan's own flat points (the shadow points are appended)
    t0 = np.array([0.01, 0.0, -0.01, 0.0, 0.02, 0.0], np.float32)
    out = []
    for k in FA_DEGENERATE_SURF_CASES + FA_SURF_SKIP_CASES:
        idx = (np.arange(12) * 11 + 5 * k) % n
        for deg_in in (0, 1):
            out.append((_scaled(sharp[:5], 0.1), _scaled(flat[idx], 0.1), _scaled(cl, 0.1), _scaled(sl, 0.1),
                        t0, deg_in))
    return cfg, out


# (query, offset) pairs of the fixture whose shrunk 10 + 50 query problem is degenerate
# (found by the oracle; tests/test_degenerate.py re-checks that every one of them is)
MO_DEGENERATE_CASES = ((0, 0), (0, 12), (1, 16), (1, 20), (2, 4), (2, 8), (3, 12), (3, 28))
# and a few that are not (the same shrunk scenes): the mix exercises both branches in one batch
MO_REGULAR_CASES = ((1, 0), (2, 0))


def mo_shrunk_problem(z, i, off):
    tr = z[f"q{i}_true"][3:]
    cm = np.array(z["corner_map"], np.float32, copy=True)
    cm[:, :3] = (cm[:, :3] - tr) * np.float32(0.05)
    sm = np.array(z["surf_map"], np.float32, copy=True)
    sm[:, :3] = (sm[:, :3] - tr) * np.float32(0.05)
    cq, sq = _scaled(z[f"q{i}_corner"], 0.05), _scaled(z[f"q{i}_surf"], 0.05)
    init = np.array(z[f"q{i}_init"], np.float32, copy=True)
    init[3:] = (init[3:] - tr) * np.float32(0.05)
    ci = (np.arange(10) * 13 + off) % len(cq)
    si = (np.arange(50) * 17 + off) % len(sq)
    return cq[ci], sq[si], cm, sm, init


def mo_degenerate_problems(regular=False):
    """[(corner_q, surf_q, corner_map, surf_map, pose0)]: the committed fixture shrunk 20x around a
    query's sensor with 10 corner / 50 surf queries (MO_DEGENERATE_CASES, + MO_REGULAR_CASES)."""
    z = np.load(FIX)
    cases = MO_DEGENERATE_CASES + (MO_REGULAR_CASES if regular else ())
    return [mo_shrunk_problem(z, i, off) for i, off in cases]


def zero_curvature_scan(seed, centers=(900,), q=2.0 ** -8):
    """A 4-fold symmetric VLP-16 scan (synth.make_symmetric_scan) whose lowest ring (-15 deg) meets
    the ground, around each raw column c in `centers`, on the line through the ground point P at c
    perpendicular to its ray: the points at columns c + 5m, m = -5..5 — consecutive in the
    segmented cloud, since ground cells enter it every 5th column (IP:809-812) — are P +- w_m with P
    and w_m on a 2^-8 m grid (z too), so the neighbour sums of calculateSmoothnessOurs (FA:826-835)
    cancel exactly at P: an exact zero curvature in ring 0's sort range per centre. Those tie with
    the phantom entry cloudSmoothness[4] = {0, ind}, and libstdc++'s order of equal values decides
    which index position 4 carries into the next frame (its flat loop visits that entry first)."""
    from llsr import synth
    pts = synth.make_symmetric_scan(seed)
    W, Hh = 1800, 16
    res = 2.0 * np.pi / W
    z = np.round(-1.3 / q) * q
    rho = -z / np.tan(np.deg2rad(15.0))
    for c in centers:
        phi = (W / 2 - c) * res
        P = np.round(np.array([rho * np.cos(phi), rho * np.sin(phi)]) / q) * q
        u = np.array([np.sin(phi), -np.cos(phi)])  # along increasing raw column (decreasing phi)
        for m in range(-5, 6):
            w = np.round(rho * np.tan(5 * abs(m) * res) * u / q) * q
            xy = P + np.sign(m) * w
            pts[((c + 5 * m) % W) * Hh + 0, :3] = (np.float32(xy[0]), np.float32(xy[1]), np.float32(z))
    return pts
