"""GPU parity of the scan-to-map LM (MapOptimization::scan2MapOptimization, MO:1572-1610).

HIP path through the C-ABI (llsr_scan2map / llsr_scan2map_batch) against the oracle
(oracle/oracle_mo.cpp) on the committed ~100k-point map fixture (13.0k corner + 87.3k surf) (tests/golden/make_mo_fixture.py).

The bar is bit-exactness: the correspondences and Jacobian rows repeat the reference's float /
double operations one for one, and the normal equations are summed in the order of the
reference's Eigen 3.3.7 build (matAt * matA per GEMM depth block, rows 4-5 x columns 0-3 through
gebp's four-accumulator path, matAt * matB and CF_all left to right; k_s2m_reduce), so the final
pose, iteration count, matX0, min_lambda, cf_mean and correspondence counts equal the oracle's.
"""
import os

import numpy as np
import pytest

import oracle_py
from llsr import Pipeline, _abi, default_config

pytestmark = pytest.mark.gpu

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mo_map_vlp16.npz")


@pytest.fixture(scope="module")
def fix():
    return np.load(FIX)


def _cfg(mode):
    cfg = default_config("vlp16")
    cfg.mode = mode
    return cfg


def _inputs(fix, i):
    return fix[f"q{i}_corner"], fix[f"q{i}_surf"], fix["corner_map"], fix["surf_map"], fix[f"q{i}_init"]


@pytest.mark.parametrize("mode", [_abi.LLSR_MODE_LM_APPLIED, _abi.LLSR_MODE_FAITHFUL])
def test_scan2map_matches_oracle(require_gpu, fix, mode):
    cfg = _cfg(mode)
    pipe = Pipeline(cfg)
    errs = []
    queries = range(int(fix["n_queries"])) if mode == _abi.LLSR_MODE_LM_APPLIED else [0, 2]
    for i in queries:
        args = _inputs(fix, i)
        g = pipe.scan2map(*args)
        o = oracle_py.scan2map(cfg, *args)
        tag = f"query {i} mode {mode}"
        for k in ("pose", "matX0", "min_lambda", "cf_mean", "iterations", "converged", "degenerate",
                  "n_corner_corr", "n_surf_corr"):
            if not np.array_equal(np.asarray(g[k]), np.asarray(o[k])):
                errs.append(f"{tag}: {k} {g[k]} vs {o[k]}")
        if mode == _abi.LLSR_MODE_FAITHFUL:
            np.testing.assert_array_equal(g["pose"], args[4])
    pipe.close()
    assert not errs, "\n".join(errs)


def test_scan2map_batch_matches_single(require_gpu, fix):
    """Device-resident batch of ragged problems == the oracle per problem."""
    import torch
    cfg = _cfg(_abi.LLSR_MODE_LM_APPLIED)
    nq = int(fix["n_queries"])
    probs = []
    for p in range(6):
        cq, sq, cm, sm, pose = _inputs(fix, p % nq)
        if p >= nq:  # ragged: fewer queries, a cropped map, another start pose
            cq, sq, cm, sm = cq[: len(cq) // 2], sq[: 2 * len(sq) // 3], cm[: 3 * len(cm) // 4], sm
            pose = pose + np.float32(0.01)
        probs.append((cq, sq, cm, sm, pose.astype(np.float32)))

    def pack(k):
        arrs = [pr[k] for pr in probs]
        off = np.zeros(len(arrs) + 1, np.int64)
        off[1:] = np.cumsum([len(a) for a in arrs])
        return torch.from_numpy(np.concatenate(arrs)).cuda(), torch.from_numpy(off).cuda()

    P = len(probs)
    (cq, cqo), (sq, sqo), (cm, cmo), (sm, smo) = (pack(k) for k in range(4))
    pose = torch.from_numpy(np.stack([pr[4] for pr in probs])).cuda()
    rep = torch.zeros(P * C_sizeof_report() // 4, dtype=torch.float32, device="cuda")
    pipe = Pipeline(cfg)
    pipe.scan2map_reserve(P, max(len(pr[2]) for pr in probs), max(len(pr[3]) for pr in probs),
                          max(len(pr[0]) for pr in probs), max(len(pr[1]) for pr in probs))
    torch.cuda.synchronize()
    pipe.scan2map_batch(dict(corner_q=cq.data_ptr(), corner_q_off=cqo.data_ptr(), surf_q=sq.data_ptr(),
                             surf_q_off=sqo.data_ptr(), corner_map=cm.data_ptr(), corner_map_off=cmo.data_ptr(),
                             surf_map=sm.data_ptr(), surf_map_off=smo.data_ptr(), pose=pose.data_ptr(),
                             report=rep.data_ptr()), P)
    torch.cuda.synchronize()
    poses = pose.cpu().numpy()
    reps = _reports(rep.cpu().numpy(), P)
    pipe.close()
    for p, pr in enumerate(probs):
        o = oracle_py.scan2map(cfg, *pr)
        np.testing.assert_array_equal(poses[p], o["pose"])
        np.testing.assert_array_equal(reps[p].pose[:], poses[p])
        assert reps[p].iterations == o["iterations"] and reps[p].converged == o["converged"], p
        assert (reps[p].n_corner_corr, reps[p].n_surf_corr) == (o["n_corner_corr"], o["n_surf_corr"]), p


def C_sizeof_report():
    import ctypes
    return ctypes.sizeof(_abi.LmReport)


def _reports(buf, P):
    import ctypes
    raw = buf.tobytes()
    n = ctypes.sizeof(_abi.LmReport)
    return [_abi.LmReport.from_buffer_copy(raw[p * n:(p + 1) * n]) for p in range(P)]


def test_scan2map_guard_and_empty(require_gpu, fix):
    cfg = _cfg(_abi.LLSR_MODE_LM_APPLIED)
    pipe = Pipeline(cfg)
    cq, sq, cm, sm, pose = _inputs(fix, 0)
    # MO:1573 guard: <= 10 corner map points -> no optimisation, pose untouched
    g = pipe.scan2map(cq, sq, cm[:10], sm, pose)
    assert g["iterations"] == 0 and np.array_equal(g["pose"], pose)
    # no queries at all: every iteration has < 50 correspondences -> iterCountThres, no update
    g = pipe.scan2map(cq[:0], sq[:0], cm, sm, pose)
    o = oracle_py.scan2map(cfg, cq[:0], sq[:0], cm, sm, pose)
    assert g["iterations"] == o["iterations"] == cfg.iterCountThres
    assert np.array_equal(g["pose"], pose) and not g["converged"]
    # corners only
    g = pipe.scan2map(cq, sq[:0], cm, sm, pose)
    o = oracle_py.scan2map(cfg, cq, sq[:0], cm, sm, pose)
    assert np.array_equal(g["pose"], o["pose"]) and g["iterations"] == o["iterations"]
    pipe.close()


def test_scan2map_capacity_error(require_gpu, fix):
    import torch
    from llsr import LlsrError
    cfg = _cfg(_abi.LLSR_MODE_LM_APPLIED)
    cq, sq, cm, sm, pose = _inputs(fix, 0)
    pipe = Pipeline(cfg)
    pipe.scan2map_reserve(1, 100, 100, 10, 10)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in
         dict(cq=cq, sq=sq, cm=cm, sm=sm, pose=pose[None]).items()}
    offs = {k: torch.tensor([0, len(v)], dtype=torch.int64).cuda() for k, v in dict(cq=cq, sq=sq, cm=cm, sm=sm).items()}
    rep = torch.zeros(64, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    with pytest.raises(LlsrError):
        pipe.scan2map_batch(dict(corner_q=t["cq"].data_ptr(), corner_q_off=offs["cq"].data_ptr(),
                                 surf_q=t["sq"].data_ptr(), surf_q_off=offs["sq"].data_ptr(),
                                 corner_map=t["cm"].data_ptr(), corner_map_off=offs["cm"].data_ptr(),
                                 surf_map=t["sm"].data_ptr(), surf_map_off=offs["sm"].data_ptr(),
                                 pose=t["pose"].data_ptr(), report=rep.data_ptr()), 1)
    pipe.close()


@pytest.mark.parametrize("mode", [_abi.LLSR_MODE_LM_APPLIED, _abi.LLSR_MODE_FAITHFUL])
def test_scan2map_degenerate(require_gpu, mode):
    """The degenerate branch (MO:1507-1537: every eigenvalue of the 6x6 AtA below 100, matP =
    matV.inverse() * matV2 through PartialPivLU) and the shrunk scenes' regular, ill-conditioned
    problems (tests/_scenes.py, smallest eigenvalue just above the threshold): bit-exact, like
    every other problem, now that AtA is summed in Eigen's order."""
    import _scenes
    cfg = _cfg(mode)
    pipe = Pipeline(cfg)
    errs = []
    for k, pr in enumerate(_scenes.mo_degenerate_problems(regular=True)):
        g = pipe.scan2map(*pr)
        o = oracle_py.scan2map(cfg, *pr)
        for key in ("pose", "degenerate", "converged", "iterations", "n_corner_corr", "n_surf_corr", "min_lambda"):
            if not np.array_equal(np.asarray(g[key]), np.asarray(o[key])):
                errs.append(f"problem {k}: {key} {g[key]} vs {o[key]}")
        if o["degenerate"] and not np.array_equal(g["pose"], pr[4]):
            errs.append(f"problem {k}: a degenerate problem moved the pose")
    pipe.close()
    assert not errs, "\n".join(errs)


def test_scan2map_more_depth_blocks_than_lds(require_gpu):
    """A problem with ~50k correspondences: Eigen's GEMM splits matAt * matA into 74 depth blocks of
    kc = 680 rows, more than the 64 k_s2m_solve keeps in LDS; the rest go through the
    problem's spill rows. Bit-exact against the oracle, no LLSR_ERANGE."""
    rng = np.random.default_rng(17)
    g = np.arange(-60.0, 60.0, 0.35, dtype=np.float32)
    xx, yy = np.meshgrid(g, g, indexing="ij")
    surf_map = np.stack([xx.ravel(), yy.ravel(), rng.normal(0, 0.01, xx.size), np.zeros(xx.size)], 1)
    surf_map = surf_map.astype(np.float32)
    n = 50000
    surf_q = np.stack([rng.uniform(-55, 55, n), rng.uniform(-55, 55, n), rng.normal(0, 0.02, n),
                       np.zeros(n)], 1).astype(np.float32)
    corner_map = np.stack([np.full(40, 5.0), np.full(40, 5.0), np.linspace(0, 4, 40), np.zeros(40)], 1)
    corner_map = corner_map.astype(np.float32)
    corner_q = np.zeros((0, 4), np.float32)
    pose0 = np.array([0.01, -0.02, 0.015, 0.1, 0.05, -0.2], np.float32)
    cfg = _cfg(_abi.LLSR_MODE_LM_APPLIED)
    cfg.iterCountThres = 3
    pipe = Pipeline(cfg)
    gm = pipe.scan2map(corner_q, surf_q, corner_map, surf_map, pose0)
    om = oracle_py.scan2map(cfg, corner_q, surf_q, corner_map, surf_map, pose0)
    pipe.close()
    assert om["n_surf_corr"] > 44000, om["n_surf_corr"]  # > 64 depth blocks of 680 rows
    for k in ("pose", "matX0", "min_lambda", "cf_mean", "iterations", "converged", "degenerate",
              "n_corner_corr", "n_surf_corr"):
        assert np.array_equal(np.asarray(gm[k]), np.asarray(om[k])), (k, gm[k], om[k])
