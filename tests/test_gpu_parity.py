"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the same inputs.

Bit-exact for labels / indices / clouds (see _compare.py for the bar). Sequences of scans run
through one handle so the FeatureAssociation carry-over state (picked / cloudLabel arrays,
phantom smoothness entry) is exercised exactly as in the reference's long-running node.
"""
import numpy as np
import pytest

from _compare import compare
from llsr import Pipeline, default_config, synth
import oracle_py

pytestmark = pytest.mark.gpu


def _run_pair(lidar, horizontal, seeds):
    cfg = default_config(lidar, horizontal)
    pipe = Pipeline(cfg, max_points=2 * cfg.num_vertical_scans * cfg.num_horizontal_scans)
    ora = oracle_py.Oracle(cfg)
    failures = []
    for s in seeds:
        pts = synth.make_scan(s, lidar)
        g = pipe.process_scan(pts)
        o = ora.process(pts)
        errs = compare(g, o)
        if errs:
            failures.append((s, errs))
    pipe.close()
    return failures


def test_vlp16_sequence_bit_exact(require_gpu):
    failures = _run_pair("vlp16", None, [1, 2, 3, 70, 71])
    assert not failures, "\n".join(f"seed {s}:\n  " + "\n  ".join(e) for s, e in failures)


def test_hdl64e_bit_exact(require_gpu):
    failures = _run_pair("hdl64e", 2048, [5, 6])
    assert not failures, "\n".join(f"seed {s}:\n  " + "\n  ".join(e) for s, e in failures)


def test_batch_matches_oracle_per_slot(require_gpu):
    import torch
    cfg = default_config("vlp16")
    B = 6
    pts, off = synth.make_batch(B, "vlp16", distinct=3, seed0=11)
    pipe = Pipeline(cfg, max_batch=B, max_points=40000)
    d_pts = torch.from_numpy(pts).cuda()
    d_off = torch.from_numpy(off).cuda()
    torch.cuda.synchronize()
    oracles = [oracle_py.Oracle(cfg) for _ in range(B)]
    for rep in range(2):  # second batch exercises per-slot carry-over state
        pipe.process_batch(d_pts.data_ptr(), d_off.data_ptr(), B)
        for b in range(B):
            o = oracles[b].process(pts[off[b]:off[b + 1]])
            errs = compare(pipe.fetch(b), o)
            assert not errs, f"rep {rep} slot {b}:\n  " + "\n  ".join(errs)
    pipe.close()


def _edge_inputs():
    rng = np.random.default_rng(5)
    base = synth.make_scan(3, "vlp16")
    finite = base[np.isfinite(base[:, 0])]
    dup = np.concatenate([finite[:5000], finite[:5000] * np.float32(1.001)], axis=0)  # collisions
    tiny = finite[:40]
    allnan = np.full((100, 4), np.nan, dtype=np.float32)
    origin = np.zeros((10, 4), dtype=np.float32)  # range 0 -> dropped (IP:333)
    shuffled = finite[rng.permutation(finite.shape[0])]
    return {"empty": np.zeros((0, 4), np.float32), "allnan": allnan, "tiny": tiny,
            "collisions": dup, "origin": origin, "shuffled": shuffled}


@pytest.mark.parametrize("case", ["empty", "allnan", "tiny", "collisions", "origin", "shuffled"])
def test_edge_cases(require_gpu, case):
    cfg = default_config("vlp16")
    pts = _edge_inputs()[case]
    pipe = Pipeline(cfg, max_points=40000)
    ora = oracle_py.Oracle(cfg)
    g, o = pipe.process_scan(pts), ora.process(pts)
    errs = compare(g, o)
    pipe.close()
    assert not errs, f"{case}:\n  " + "\n  ".join(errs)
