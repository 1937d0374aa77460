"""Probe: does the order of a problem's queries change the scan-to-map LM's speed? The bench's
configs[2] leg (P problems on the 100k-point fixture map, lm_applied) with each problem's corner /
surf queries in the fixture's order and, for comparison, sorted by a Morton code of their 2 m cells
(a rigid pose keeps neighbourhoods, so the scan-frame cells group the map cells the kNN-5 reads).
Results differ between orders (LMOptimization sums the rows in query order); only the timing is
compared.   python scripts/s2m_order_probe.py [P] [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-sr_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from llsr import Pipeline, _abi, default_config  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 256
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5


def morton_order(q, cell=2.0):
    c = np.floor(q[:, :3] / cell).astype(np.int64)
    c -= c.min(0)
    key = np.zeros(len(q), np.int64)
    for bit in range(10):
        for a in range(3):
            key |= ((c[:, a] >> bit) & 1) << (3 * bit + a)
    return np.argsort(key, kind="stable")


def run(order):
    z = np.load(os.path.join(REPO, "tests", "golden", "mo_map_vlp16.npz"))
    nq = int(z["n_queries"])
    cfg = default_config("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    cm, sm = z["corner_map"], z["surf_map"]
    rng = np.random.default_rng(99)
    probs = []
    for p in range(P):
        q = p % nq
        pose = z[f"q{q}_true"] + np.concatenate([rng.uniform(-0.05, 0.05, 3), rng.uniform(-0.2, 0.2, 3)])
        c, s = z[f"q{q}_corner"], z[f"q{q}_surf"]
        if order == "spatial":
            c, s = c[morton_order(c)], s[morton_order(s)]
        probs.append((np.ascontiguousarray(c), np.ascontiguousarray(s), cm, sm, pose.astype(np.float32)))

    def pack(k):
        arrs = [pr[k] for pr in probs]
        off = np.zeros(P + 1, np.int64)
        off[1:] = np.cumsum([len(a) for a in arrs])
        return torch.from_numpy(np.concatenate(arrs)).cuda(), torch.from_numpy(off).cuda()

    (cq, cqo), (sq, sqo), (dcm, cmo), (dsm, smo) = (pack(k) for k in range(4))
    pose0 = torch.from_numpy(np.stack([pr[4] for pr in probs])).cuda()
    pose = pose0.clone()
    import ctypes
    rep = torch.zeros((P, ctypes.sizeof(_abi.LmReport) // 4), dtype=torch.float32, device="cuda")
    pipe = Pipeline(cfg)
    pipe.scan2map_reserve(P, len(cm), len(sm), max(len(pr[0]) for pr in probs), max(len(pr[1]) for pr in probs))
    ptrs = dict(corner_q=cq.data_ptr(), corner_q_off=cqo.data_ptr(), surf_q=sq.data_ptr(),
                surf_q_off=sqo.data_ptr(), corner_map=dcm.data_ptr(), corner_map_off=cmo.data_ptr(),
                surf_map=dsm.data_ptr(), surf_map_off=smo.data_ptr(), pose=pose.data_ptr(), report=rep.data_ptr())
    stream = torch.cuda.Stream()

    def step():
        with torch.cuda.stream(stream):
            pose.copy_(pose0)
            pipe.scan2map_batch(ptrs, P, stream.cuda_stream)

    step()
    torch.cuda.synchronize()
    pipe.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(STEPS):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = pipe.scan2map_stats()
    pipe.close()
    return {"order": order, "problems_per_s": round(P * STEPS / el, 1), "ms_per_step": round(el / STEPS * 1e3, 3),
            "grid_ms": round(st["grid_ms"] / STEPS, 4), "iterate_ms": round(st["iterate_ms"] / STEPS, 4),
            "iter_launches": st["iteration_launches"] / STEPS}


for o in ("input", "spatial", "input", "spatial"):
    print(run(o), flush=True)
