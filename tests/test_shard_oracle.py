"""CPU tests of the split-correspondence scan-to-map: the int64 fixed-point
normal equations make the result independent of how the correspondences are split over ranks.

* the oracle's split statement (oracle_mo.cpp oracle_s2m_shard_*) gives bit-identical reports
  for 1, 2, 3 and 5 simulated ranks, within the pose tolerance of the float restatement;
* the product driver llsr.dist.sharded_scan2map over a real 2-process gloo group (MASTER
  127.0.0.1) reproduces the single-process result bit for bit, on every rank.
The device's split kernels are checked against the same statement in tests/test_gpu_shard.py.
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

import oracle_py
from llsr import _abi
from llsr.dist import shard_range

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mo_map_vlp16.npz")
POSE_TOL = 1e-4


@pytest.fixture(scope="module")
def fix():
    return np.load(FIX)


def _probs(fix, queries):
    return [(fix[f"q{i}_corner"], fix[f"q{i}_surf"], fix["corner_map"], fix["surf_map"], fix[f"q{i}_init"])
            for i in queries]


def _cfg(mode, iters=200):
    cfg = _abi.config_for("vlp16")
    cfg.mode = mode
    cfg.iterCountThres = iters
    return cfg


def _same(a, b):
    return all(np.array_equal(np.asarray(a[k]), np.asarray(b[k])) for k in a if k != "ms")


@pytest.mark.parametrize("mode,iters", [(_abi.LLSR_MODE_LM_APPLIED, 200), (_abi.LLSR_MODE_FAITHFUL, 12)])
def test_split_invariance_and_float_tolerance(fix, mode, iters):
    cfg = _cfg(mode, iters)
    probs = _probs(fix, [0, 1])
    ref = oracle_py.shard_run_local(cfg, probs, 1)
    for W in (2, 3, 5):
        res = oracle_py.shard_run_local(cfg, probs, W)
        for p in range(len(probs)):
            assert _same(res[p], ref[p]), (W, p)
    for p, pr in enumerate(probs):
        f = oracle_py.scan2map(cfg, *pr)
        r = ref[p]
        assert np.abs(r["pose"] - f["pose"]).max() <= POSE_TOL
        assert r["iterations"] == f["iterations"] and r["converged"] == f["converged"]
        # same correspondences; only the rounding of the summed terms differs
        assert (r["n_corner_corr"], r["n_surf_corr"]) == (f["n_corner_corr"], f["n_surf_corr"])
        np.testing.assert_allclose(r["matX0"], f["matX0"], rtol=1e-4, atol=1e-6)
        if mode == _abi.LLSR_MODE_FAITHFUL:
            np.testing.assert_array_equal(r["pose"], pr[4])


def test_fixed_point_rounding_is_exact_integer_sum():
    from llsr import _abi as a  # noqa: F401
    # the words are plain integer sums: a split of the terms in any grouping adds to the same words
    rng = np.random.default_rng(0)
    terms = (rng.normal(0, 300, 5000).astype(np.float32).astype(np.float64) * 2**30).round().astype(np.int64)
    perm = rng.permutation(terms.size)
    assert terms.sum() == terms[perm].sum() == sum(terms[k::7].sum() for k in range(7))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_covers_once():
    for n in (0, 1, 7, 1024):
        for world in (1, 2, 3, 8):
            got = [i for r in range(world) for i in shard_range(n, r, world)]
            assert got == list(range(n))


def test_gloo_world2_matches_single_process(fix):
    import _dist_worker
    mode, iters, queries = _abi.LLSR_MODE_LM_APPLIED, 200, [0, 2]
    ref = oracle_py.shard_run_local(_cfg(mode, iters), _probs(fix, queries), 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker.run, args=(r, 2, port, mode, iters, queries, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in procs:
            rank, iters_run, res, t, sh = q.get(timeout=240)
            assert iters_run != "error", res
            out[rank] = (iters_run, res, t, sh)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert set(out) == {0, 1}
    for rank, (iters_run, res, t, sh) in out.items():
        assert t == pytest.approx(0.002)  # max over ranks
        assert sh == list(shard_range(10, rank, 2))
        for p, (pose, n_it, conv) in enumerate(res):
            assert np.array_equal(np.float32(pose), ref[p]["pose"]), (rank, p)
            assert n_it == ref[p]["iterations"] and conv == ref[p]["converged"]
