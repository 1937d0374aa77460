"""GPU parity of the split-correspondence scan-to-map (llsr_scan2map_shard_*).

W ranks are simulated on one device: each LM iteration runs every rank's partial kernel into its
own int64 buffer and adds the buffers (what an RCCL all-reduce delivers), then one step. The bar:
  * bit-identical reports for W = 1, 2, 3, 8 (integer sums are associative);
  * bit-identical to the oracle's CPU statement of the same split mode
    (oracle_py.shard_run_local), i.e. the device's correspondences, Jacobian terms and LM step
    equal the restatement's exactly;
  * pose within 1e-4 of the float restatement (oracle_py.scan2map).
"""
import os

import numpy as np
import pytest

import oracle_py
from llsr import Pipeline, _abi, default_config

pytestmark = pytest.mark.gpu

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mo_map_vlp16.npz")
POSE_TOL = 1e-4


def _problems(z):
    nq = int(z["n_queries"])
    probs = []
    for p in range(5):
        cq, sq, cm, sm, pose = (z[f"q{p % nq}_corner"], z[f"q{p % nq}_surf"], z["corner_map"], z["surf_map"],
                                z[f"q{p % nq}_init"])
        if p >= nq:  # ragged: fewer queries, a cropped corner map, another start pose
            cq, sq, cm = cq[: len(cq) // 2], sq[: 2 * len(sq) // 3], cm[: 3 * len(cm) // 4]
            pose = pose + np.float32(0.01)
        probs.append((cq, sq, cm, sm, np.asarray(pose, np.float32)))
    return probs


def _run_device(cfg, probs, W):
    import ctypes
    import torch
    P = len(probs)

    def pack(k):
        arrs = [np.ascontiguousarray(pr[k], np.float32) for pr in probs]
        off = np.zeros(P + 1, np.int64)
        off[1:] = np.cumsum([len(a) for a in arrs])
        return torch.from_numpy(np.concatenate(arrs)).cuda(), torch.from_numpy(off).cuda()

    (cq, cqo), (sq, sqo), (cm, cmo), (sm, smo) = (pack(k) for k in range(4))
    pose = torch.from_numpy(np.stack([pr[4] for pr in probs])).cuda()
    n = ctypes.sizeof(_abi.LmReport)
    rep = torch.zeros(P * n // 4, dtype=torch.float32, device="cuda")
    pipe = Pipeline(cfg)
    pipe.scan2map_reserve(P, max(len(pr[2]) for pr in probs), max(len(pr[3]) for pr in probs),
                          max(len(pr[0]) for pr in probs), max(len(pr[1]) for pr in probs))
    ptrs = dict(corner_q=cq.data_ptr(), corner_q_off=cqo.data_ptr(), surf_q=sq.data_ptr(), surf_q_off=sqo.data_ptr(),
                corner_map=cm.data_ptr(), corner_map_off=cmo.data_ptr(), surf_map=sm.data_ptr(),
                surf_map_off=smo.data_ptr(), pose=pose.data_ptr(), report=rep.data_ptr())
    torch.cuda.synchronize()
    # the library and torch must share one stream: a non-default one (0 = the handle's own stream)
    s = torch.cuda.Stream()
    stream = s.cuda_stream
    with torch.cuda.stream(s):
        tot = torch.zeros((P, _abi.NE_WORDS), dtype=torch.int64, device="cuda")
        part = torch.zeros_like(tot)
        pipe.scan2map_shard_begin(ptrs, P, stream)
        for it in range(cfg.iterCountThres):
            tot.zero_()
            for r in range(W):
                pipe.scan2map_shard_partial(r, W, part.data_ptr(), stream)
                tot += part
            if pipe.scan2map_shard_step(tot.data_ptr(), True, stream) == 0:
                break
        pipe.scan2map_shard_end(stream)
    torch.cuda.synchronize()
    raw = rep.cpu().numpy().tobytes()
    out = []
    for p in range(P):
        d = _abi.LmReport.from_buffer_copy(raw[p * n:(p + 1) * n]).as_dict()
        out.append(d)
    poses = pose.cpu().numpy()
    pipe.close()
    for p in range(P):
        np.testing.assert_array_equal(out[p]["pose"], poses[p])
    return out


def _same(a, b):
    return all(np.array_equal(np.asarray(a[k]), np.asarray(b[k])) for k in a if k != "ms")


@pytest.mark.parametrize("mode,iters", [(_abi.LLSR_MODE_LM_APPLIED, 200), (_abi.LLSR_MODE_FAITHFUL, 16)])
def test_shard_split_invariant_and_bit_exact_vs_oracle(require_gpu, mode, iters):
    z = np.load(FIX)
    cfg = default_config("vlp16")
    cfg.mode = mode
    cfg.iterCountThres = iters
    probs = _problems(z)
    ora = oracle_py.shard_run_local(cfg, probs, 1)
    errs = []
    for W in (1, 2, 3, 8):
        dev = _run_device(cfg, probs, W)
        for p in range(len(probs)):
            if not _same(dev[p], ora[p]):
                errs.append(f"W={W} problem {p}: device {dev[p]} vs oracle split statement {ora[p]}")
    for p, pr in enumerate(probs):
        f = oracle_py.scan2map(cfg, *pr)
        if np.abs(ora[p]["pose"] - f["pose"]).max() > POSE_TOL:
            errs.append(f"problem {p}: split pose {ora[p]['pose']} vs float {f['pose']}")
    assert not errs, "\n".join(errs)


def test_shard_api_errors(require_gpu):
    import torch
    from llsr import LlsrError
    pipe = Pipeline(default_config("vlp16"))
    ne = torch.zeros((1, _abi.NE_WORDS), dtype=torch.int64, device="cuda")
    with pytest.raises(LlsrError):
        pipe.scan2map_shard_partial(0, 1, ne.data_ptr())  # no open batch
    with pytest.raises(LlsrError):
        pipe.scan2map_shard_step(ne.data_ptr(), True)
    pipe.close()


def test_shard_degenerate_bit_exact_vs_oracle(require_gpu):
    """Split mode on degenerate + regular shrunk problems (tests/_scenes.py): the device's LM step
    (QR, 6x6 eigen, PartialPivLU inverse, projection — llsr_eigen.h) equals the oracle's independent
    restatement (oracle_eigen.h) bit for bit, for W = 1 and 3."""
    import _scenes
    cfg = default_config("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    probs = _scenes.mo_degenerate_problems(regular=True)
    ora = oracle_py.shard_run_local(cfg, probs, 1)
    assert sum(o["degenerate"] for o in ora) == len(_scenes.MO_DEGENERATE_CASES)
    errs = []
    for W in (1, 3):
        dev = _run_device(cfg, probs, W)
        for p in range(len(probs)):
            if not _same(dev[p], ora[p]):
                errs.append(f"W={W} problem {p}: device {dev[p]} vs oracle split statement {ora[p]}")
    assert not errs, "\n".join(errs)
