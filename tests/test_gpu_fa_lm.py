"""GPU parity of the scan-to-scan LM (FeatureAssociation::updateTransformation, FA:2505-2535).

HIP path (llsr_scan2scan / llsr_scan2scan_batch) against the oracle (oracle/oracle_fa_lm.cpp)
on consecutive synthetic VLP-16 scans: the inputs are the oracle's own feature-stage outputs
(bit-exact with the HIP feature stage, tests/test_gpu_parity.py) assembled as
runFeatureAssociation does (oracle_py.fa_lm_inputs). The device sums the normal equations in
the oracle's correspondence order, so the bar is bit-exact: transformCur, iteration counts,
correspondence counts and the degeneracy flag all equal.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_py
from llsr import Pipeline, _abi, default_config, lib, shadow_points, synth

pytestmark = pytest.mark.gpu


def _pairs(lidar, seeds, horizontal=None, motion=True):
    """Consecutive frames of a moving sensor (synth.sensor_attitude: z, roll, pitch and yaw change
    from frame to frame, so the surf step iterates, FA:1846-2010)."""
    cfg = default_config(lidar, horizontal)
    ora = oracle_py.Oracle(cfg)
    prev = ora.process(synth.make_scan(seeds[0], lidar, motion=motion))
    out = []
    for s in seeds[1:]:
        cur = ora.process(synth.make_scan(s, lidar, motion=motion))
        out.append(oracle_py.fa_lm_inputs(prev, cur))
        prev = cur
    return cfg, out


def _same(g, o):
    errs = []
    if not np.array_equal(g["transform_cur"], o["transform_cur"]):
        errs.append(f"transform_cur {g['transform_cur']} vs {o['transform_cur']} "
                    f"(max |d| {np.abs(g['transform_cur'] - o['transform_cur']).max():.3g})")
    for k in ("surf_iterations", "corner_iterations", "n_surf_corr", "n_corner_corr", "degenerate", "skipped"):
        if g[k] != o[k]:
            errs.append(f"{k} {g[k]} vs {o[k]}")
    return errs


def test_shadow_points_match_oracle(require_gpu):
    np.testing.assert_array_equal(shadow_points(), oracle_py.shadow_points())


@pytest.mark.parametrize("lidar,seeds,horizontal", [("vlp16", [1, 2, 3, 4, 5, 6, 7, 70], None),
                                                    ("hdl64e", [5, 6, 7, 8], 2048)])
def test_scan2scan_bit_exact(require_gpu, lidar, seeds, horizontal):
    """Every surf iteration past the first is covered: the kNN refresh every 5th iteration and the
    parked indices in between (FA:1707-1803), the iterCount >= 5 weighting (FA:1825-1830) and the
    surf update of pitch / roll / vertical translation (FA:2001-2003) — at least one pair per lidar
    runs the surf step for >= 6 iterations (asserted on the oracle's count)."""
    cfg, pairs = _pairs(lidar, seeds, horizontal)
    pipe = Pipeline(cfg)
    errs, surf_its = [], []
    t = np.zeros(6, np.float32)
    for k, (sharp, flat, cl, sl) in enumerate(pairs):
        g = pipe.scan2scan(sharp, flat, cl, sl, t, 0)
        o = oracle_py.scan2scan(cfg, sharp, flat, cl, sl, t, 0)
        surf_its.append(o["surf_iterations"])
        errs += [f"pair {k}: {e}" for e in _same(g, o)]
        t = o["transform_cur"] * np.float32(0.5)  # a non-zero initial guess for the next pair
    pipe.close()
    assert not errs, "\n".join(errs)
    assert max(surf_its) >= 6, f"no pair iterates the surf step: {surf_its}"


def test_scan2scan_batch_and_skip(require_gpu):
    import torch
    cfg, pairs = _pairs("vlp16", [11, 12, 13, 14, 15])
    assert max(oracle_py.scan2scan(cfg, *pr, np.zeros(6, np.float32), 0)["surf_iterations"] for pr in pairs) >= 6
    # problem 4: a last corner cloud below the FA:2506 guard -> skipped, transform untouched
    pairs.append((pairs[0][0], pairs[0][1], pairs[0][2][:9], pairs[0][3]))
    P = len(pairs)
    t0 = np.random.default_rng(3).uniform(-0.01, 0.01, (P, 6)).astype(np.float32)

    def pack(k):
        arrs = [pr[k] for pr in pairs]
        off = np.zeros(P + 1, np.int64)
        off[1:] = np.cumsum([len(a) for a in arrs])
        return torch.from_numpy(np.concatenate(arrs)).cuda(), torch.from_numpy(off).cuda()

    (sh, sho), (fl, flo), (cl, clo), (sl, slo) = (pack(k) for k in range(4))
    tc = torch.from_numpy(t0.copy()).cuda()
    deg = torch.zeros(P, dtype=torch.int32).cuda()
    import ctypes
    rep = torch.zeros(P * ctypes.sizeof(_abi.S2SReport) // 4, dtype=torch.float32).cuda()
    pipe = Pipeline(cfg)
    pipe.scan2scan_reserve(P, *(max(len(pr[k]) for pr in pairs) for k in range(4)))
    torch.cuda.synchronize()
    pipe.scan2scan_batch(dict(sharp=sh.data_ptr(), sharp_off=sho.data_ptr(), flat=fl.data_ptr(), flat_off=flo.data_ptr(),
                              corner_last=cl.data_ptr(), corner_last_off=clo.data_ptr(), surf_last=sl.data_ptr(),
                              surf_last_off=slo.data_ptr(), transform_cur=tc.data_ptr(),
                              is_degenerate=deg.data_ptr(), report=rep.data_ptr()), P)
    pipe.scan2scan_check()
    tg = tc.cpu().numpy()
    raw = rep.cpu().numpy().tobytes()
    n = ctypes.sizeof(_abi.S2SReport)
    pipe.close()
    for p, pr in enumerate(pairs):
        o = oracle_py.scan2scan(cfg, *pr, t0[p], 0)
        g = _abi.S2SReport.from_buffer_copy(raw[p * n:(p + 1) * n]).as_dict()
        g["transform_cur"] = tg[p]
        assert not _same(g, o), (p, _same(g, o))
    assert _abi.S2SReport.from_buffer_copy(raw[(P - 1) * n:P * n]).skipped == 1
    np.testing.assert_array_equal(tg[P - 1], t0[P - 1])


def test_scan2scan_capacity_error(require_gpu):
    import torch
    from llsr import LlsrError
    cfg, pairs = _pairs("vlp16", [21, 22])
    sharp, flat, cl, sl = pairs[0]
    pipe = Pipeline(cfg)
    pipe.scan2scan_reserve(1, 8, 8, 8, 8)
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (sharp, flat, cl, sl)]
    o = [torch.tensor([0, len(a)], dtype=torch.int64).cuda() for a in (sharp, flat, cl, sl)]
    tc = torch.zeros(6).cuda()
    deg = torch.zeros(1, dtype=torch.int32).cuda()
    rep = torch.zeros(64).cuda()
    torch.cuda.synchronize()
    pipe.scan2scan_batch(dict(sharp=d[0].data_ptr(), sharp_off=o[0].data_ptr(), flat=d[1].data_ptr(),
                              flat_off=o[1].data_ptr(), corner_last=d[2].data_ptr(), corner_last_off=o[2].data_ptr(),
                              surf_last=d[3].data_ptr(), surf_last_off=o[3].data_ptr(), transform_cur=tc.data_ptr(),
                              is_degenerate=deg.data_ptr(), report=rep.data_ptr()), 1)
    with pytest.raises(LlsrError):
        pipe.scan2scan_check()
    pipe.close()


def test_scan2scan_degenerate_bit_exact(require_gpu):
    """The degenerate branch (FA:1959-1990: all eigenvalues of the corner phase's AtA below 10,
    matP = matV.inverse() * matV2 with the cofactor inverse) on shrunk scenes (tests/_scenes.py):
    device == oracle bit for bit, including the flag."""
    import _scenes
    cfg, pairs = _scenes.fa_degenerate_pairs()
    pipe = Pipeline(cfg)
    errs, n_deg = [], 0
    for k, (sharp, flat, cl, sl, t0) in enumerate(pairs):
        g = pipe.scan2scan(sharp, flat, cl, sl, t0, 0)
        o = oracle_py.scan2scan(cfg, sharp, flat, cl, sl, t0, 0)
        n_deg += o["degenerate"]
        errs += [f"pair {k}: {e}" for e in _same(g, o)]
    pipe.close()
    assert n_deg >= 4
    assert not errs, "\n".join(errs)


def test_scan2scan_degenerate_surf_bit_exact(require_gpu):
    """The surf step's degenerate branch (FA:1959-1996): shrunk scenes with 12 flat queries whose
    iteration-0 AtA has every eigenvalue below 10 (matP = matV.inverse() * 0, the pose stays, the
    step stops: surf_iterations 0 with the flag set), and scenes with fewer than 10 surf
    correspondences, where every surf iteration is skipped (FA:2516) and a carried-in isDegenerate
    survives into the corner step (5 sharp points: skipped too, so the flag reported is the surf
    step's). matP at iteration >= 1 after a degenerate iteration 0 is unreachable: a degenerate
    iteration 0 gives matX = 0, so deltaR = deltaT = 0 and the loop breaks (FA:2007-2009), and a
    skipped iteration 0 leaves the pose, hence the correspondence set, unchanged."""
    import _scenes
    cfg, cases = _scenes.fa_degenerate_surf_pairs()
    pipe = Pipeline(cfg)
    errs, n_deg, n_skip = [], 0, 0
    for k, (sharp, flat, cl, sl, t0, deg_in) in enumerate(cases):
        g = pipe.scan2scan(sharp, flat, cl, sl, t0, deg_in)
        o = oracle_py.scan2scan(cfg, sharp, flat, cl, sl, t0, deg_in)
        n_deg += o["degenerate"] and o["surf_iterations"] == 0 and o["n_surf_corr"] >= 10
        n_skip += o["surf_iterations"] == 100
        errs += [f"case {k}: {e}" for e in _same(g, o)]
        if g["is_degenerate"] != o["is_degenerate"]:
            errs.append(f"case {k}: is_degenerate {g['is_degenerate']} vs {o['is_degenerate']}")
    pipe.close()
    assert n_deg >= 3 and n_skip >= 2, (n_deg, n_skip)
    assert not errs, "\n".join(errs)


@pytest.mark.parametrize("lidar", ["vlp16", "hdl64e"])
@pytest.mark.parametrize("variant", ["twins", "shuffled", "rings_swapped"])
def test_scan2scan_surf_cloud_order(require_gpu, variant, lidar):
    """The surf tripod search reads the last cloud's order (FA:1737-1803 walk it by index): the
    device walks the cloud from the kNN hit in both directions, skipping 8-point blocks and
    64-point superblocks whose bounding boxes (k_s2s_boxes) cannot beat the current minimum and
    hold no ring stop. Twins (every point repeated in place: every distance ties) pin the tie
    rule; a shuffled cloud and one with two ring blocks swapped break the ring order the stops
    and boxes see. VLP-16 pairs run the per-lane walks (the <1024, 1024> instantiation), HDL-64E
    pairs the whole-wave walks of the large instantiations (asserted)."""
    hdl = lidar == "hdl64e"
    cfg, pairs = _pairs(lidar, [41, 42] if hdl else [31, 32, 33], 2048 if hdl else None)
    pipe = Pipeline(cfg)
    variant_of = lib().llsr_debug_s2s_variant
    variant_of.restype, variant_of.argtypes = C.c_int32, [C.c_void_p]
    errs = []
    rng = np.random.default_rng(7)
    for k, (sharp, flat, cl, sl) in enumerate(pairs):
        if variant == "twins":
            sl = np.repeat(sl, 2, axis=0)
        elif variant == "shuffled":
            sl = sl[rng.permutation(len(sl))]
        else:
            ring = np.trunc(sl[:, 3]).astype(np.int64)
            a, b = ring == 3, ring == 9
            sl = np.concatenate([sl[ring < 3], sl[b], sl[(ring > 3) & (ring < 9)], sl[a], sl[ring > 9]])
        sl = np.ascontiguousarray(sl)
        t = np.full(6, 0.002, np.float32)
        g = pipe.scan2scan(sharp, flat, cl, sl, t, 0)
        used = variant_of(pipe._h)
        assert (used in (2560, 2048)) if hdl else used == 1024, (lidar, used)
        o = oracle_py.scan2scan(cfg, sharp, flat, cl, sl, t, 0)
        errs += [f"pair {k}: {e}" for e in _same(g, o)]
    pipe.close()
    assert not errs, "\n".join(errs)
