"""RCCL on the GPU (BASELINE.json configs[4]): the split-correspondence scan-to-map
with its per-iteration all-reduce actually executed by RCCL, at world 1 (the box has one GPU; the
collective runs all the same: ncclAllReduce of the [P][32] int64 words, in place, on the stream the
kernels use).

* The C++ path: tests/native/llsr_shard_driver (one rank over include/llsr_rccl.h:
  llsr_scan2map_rccl = shard_begin -> per iteration partial -> ncclAllReduce -> step -> end).
* The Python path: a one-rank torch.distributed "nccl" (= RCCL) group and llsr.dist.sharded_scan2map
  with force_collective, on a non-default stream shared by torch, RCCL and the library.

Bar: the reports (pose, iterations, matX0, min_lambda, cf_mean, counts) equal the oracle's CPU
statement of the split mode (oracle_py.shard_run_local) bit for bit, as the simulated-rank test does
(tests/test_gpu_shard.py).
"""
import ctypes
import os
import struct
import subprocess

import numpy as np
import pytest

import oracle_py
from llsr import Pipeline, _abi, default_config

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(REPO, "tests", "native", "llsr_shard_driver")
FIX = os.path.join(REPO, "tests", "golden", "mo_map_vlp16.npz")


def _problems():
    z = np.load(FIX)
    nq = int(z["n_queries"])
    probs = []
    for p in range(4):
        q = p % nq
        cq, sq = z[f"q{q}_corner"], z[f"q{q}_surf"]
        cm = z["corner_map"] if p < nq else z["corner_map"][: 2 * len(z["corner_map"]) // 3]
        pose = np.asarray(z[f"q{q}_init"], np.float32) + np.float32(0.005 * p)
        probs.append((cq, sq, cm, z["surf_map"], pose))
    return probs


def _same(a, b):
    return all(np.array_equal(np.asarray(a[k]), np.asarray(b[k])) for k in a if k != "ms")


def _cfg(iters):
    cfg = default_config("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    cfg.iterCountThres = iters
    return cfg


@pytest.mark.parametrize("iters,poll", [(60, 3), (50, 16), (7, 4)])
def test_cpp_driver_rccl_world1(require_gpu, tmp_path, iters, poll):
    """poll 16 does not divide 50 (nor 4 divide 7): the driver still stops at iterCountThres."""
    assert os.path.exists(DRIVER), "build it with `make -C lego-loam-sr_amd`"
    probs = _problems()
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(inp, "wb") as f:
        f.write(struct.pack("<i", len(probs)))
        for pr in probs:
            f.write(struct.pack("<4i", *(len(c) for c in pr[:4])))
            for c in pr[:4]:
                f.write(np.ascontiguousarray(c, np.float32).tobytes())
            f.write(np.ascontiguousarray(pr[4], np.float32).tobytes())
    r = subprocess.run([DRIVER, str(inp), str(out), str(_abi.LLSR_MODE_LM_APPLIED), str(iters), str(poll)],
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = out.read_bytes()
    n = ctypes.sizeof(_abi.LmReport)
    dev = [_abi.LmReport.from_buffer_copy(raw[p * n:(p + 1) * n]).as_dict() for p in range(len(probs))]
    us, it = struct.unpack("<fi", raw[len(probs) * n:len(probs) * n + 8])
    assert us > 0.0
    ora = oracle_py.shard_run_local(_cfg(iters), probs, 1)
    it_ref = max(o["iterations"] for o in ora)
    assert it_ref <= it <= min(iters, it_ref + poll - 1), (it, it_ref, iters, poll)
    errs = [f"problem {p}: {dev[p]} vs {ora[p]}" for p in range(len(probs)) if not _same(dev[p], ora[p])]
    assert not errs, "\n".join(errs)
    print(r.stdout.strip())


def test_torch_rccl_group_world1(require_gpu):
    import torch
    import torch.distributed as dist
    from llsr.dist import HipShardEngine, allreduce_latency_us, sharded_scan2map
    assert not dist.is_initialized()
    import socket
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        probs = _problems()
        P = len(probs)
        iters = 60
        cfg = _cfg(iters)

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
        ptrs = dict(corner_q=cq.data_ptr(), corner_q_off=cqo.data_ptr(), surf_q=sq.data_ptr(),
                    surf_q_off=sqo.data_ptr(), corner_map=cm.data_ptr(), corner_map_off=cmo.data_ptr(),
                    surf_map=sm.data_ptr(), surf_map_off=smo.data_ptr(), pose=pose.data_ptr(), report=rep.data_ptr())
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            eng = HipShardEngine(pipe, ptrs, P, s.cuda_stream)
            ne = eng.new_ne("cuda")
            it = sharded_scan2map(eng, ne, iters, poll=2, force_collective=True)
            lat = allreduce_latency_us(ne, reps=20)
        torch.cuda.synchronize()
        raw = rep.cpu().numpy().tobytes()
        dev = [_abi.LmReport.from_buffer_copy(raw[p * n:(p + 1) * n]).as_dict() for p in range(P)]
        pipe.close()
        ora = oracle_py.shard_run_local(cfg, probs, 1)
        errs = [f"problem {p}: {dev[p]} vs {ora[p]}" for p in range(P) if not _same(dev[p], ora[p])]
        assert not errs, "\n".join(errs)
        assert it >= max(o["iterations"] for o in ora) and lat > 0.0
        print(f"torch RCCL world 1: {it} LM iterations, all-reduce {lat:.1f} us")
    finally:
        dist.destroy_process_group()
