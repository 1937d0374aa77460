"""bench.py — scans/sec of the MI355X LeGO-LOAM-SR hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1]): synthetic VLP-16 1800x16 scans through projection + ground /
cluster segmentation (ImageProjection) + curvature / feature extraction (FeatureAssociation
feature stage), labels / feature indices bit-exact vs the CPU path. A "step" is one pass of the
hot path over one batch of B scans per GPU that is already resident in HBM.

The same JSON line carries a second measured leg, "scan2map" (BASELINE.json configs[2]): batches
of P scan-to-map problems (MapOptimization::scan2MapOptimization) against the ~100k-point local
map of tests/golden/mo_map_vlp16.npz, in lm_applied and faithful (200-iteration) mode, with the
pose delta against the CPU restatement and its own CPU baseline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

N > 1 is launched by torch.distributed.run (one rank per GPU). Scans are batch-sharded: every
rank processes its own B scans with no data-path collective (weak scaling); ranks only meet at the
barriers around the timed region and for the max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lego-loam-sr_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
VOXEL_ORDERS = {"input": 0, "pcl": 1}  # llsr.h LLSR_VOXEL_ORDER_INPUT / LLSR_VOXEL_ORDER_PCL


def kernel_bytes(name: str, c: dict, HW: int) -> float:
    """Algorithmic HBM bytes of one launch of `name` for one scan.

    c: per-scan counts  Nr raw points, N finite, S segmented, O outliers, K near, R ransac iters,
    M edges, F flats, L less-flat out, Lc less-flat candidates (~S - M - F).
    """
    N, Nr, S, K, M, F, L = c["N"], c["Nr"], c["S"], c["K"], c["M"], c["F"], c["L"]
    Lc = max(S - M - F, 0)
    return {
        "k_project": 16 * Nr + 4 * N,
        "k_gather_column": 4 * HW + 16 * N + 25 * HW,
        "k_ground_add": 2 * HW,
        "k_ground_elev_ransac": 2 * HW + 16 * N + 16 * K * (c["R"] + 2),
        "k_label": 9 * HW,
        "k_segment": 5 * HW + 53 * S + 9 * (HW - S),
        "k_fa_points": 46 * S,  # adjustDistortion + curvature: seg xyzi/range/col in, loam/curv/picked/label out
        "k_select_ring": 13 * S + 16 * Lc + 16 * L + 8 * (M + F),
        "k_fa_concat": 8 * (M + F) + 32 * L + 40 * M,
        "k_dbscan_adj": 20 * M + c.get("M2", 0) / 8,
        "k_dbscan_merge": c.get("M2", 0) / 8 + 12 * M,
    }.get(name, 0.0)


def cpu_baseline(scans: list[np.ndarray], budget_s: float) -> dict:
    """The oracle (C++ restatement of the reference CPU path, -O3, one thread) on host cores."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py
    from llsr import _abi
    ora = oracle_py.Oracle(_abi.config_for("vlp16"), pcl_voxel_order=True)  # as PCL (std::sort)
    ora.process(scans[0])  # warm-up (page-in, first-frame state)
    n, t0 = 0, time.perf_counter()
    ip_ms = fa_ms = 0.0
    while True:
        ora.process(scans[n % len(scans)])
        a, b = ora.stage_ms()
        ip_ms += a
        fa_ms += b
        n += 1
        el = time.perf_counter() - t0
        if (el >= budget_s and n >= 20) or n >= 100000:
            break
    return {"value": n / el, "unit": "scans/s", "cores": 1, "kind": "port",
            "sample": f"{n} VLP-16 scans ({len(scans)} distinct synthetic clouds, cycled) through the "
                      f"oracle IP+FA-feature path in {el:.1f} s, 1 thread",
            "ip_ms": ip_ms / n, "fa_features_ms": fa_ms / n}


def _ipfa_cpu_worker(args):
    """One process of the headline's all-core CPU baseline: the oracle IP + FA-feature path over
    the given scans (cycled) for `budget` seconds, one thread; returns (scans, busy seconds)."""
    scans, budget = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py
    from llsr import _abi
    ora = oracle_py.Oracle(_abi.config_for("vlp16"), pcl_voxel_order=True)
    ora.process(scans[0])
    n, t0 = 0, time.perf_counter()
    while True:
        ora.process(scans[n % len(scans)])
        n += 1
        el = time.perf_counter() - t0
        if el >= budget and n >= 10:
            return n, el


def cpu_baseline_all_cores(scans: list[np.ndarray], budget_s: float) -> dict:
    """all-core throughput of the headline path = independent single-threaded
    pipelines, one per host core the job is granted (16 on the GPU pool), each cycling the scans."""
    nproc = min(16, os.cpu_count() or 1)
    t1 = time.perf_counter()
    res = pool_map(_ipfa_cpu_worker, [(scans, budget_s)] * nproc, nproc)
    wall = time.perf_counter() - t1
    n = sum(r[0] for r in res)
    busy = max(r[1] for r in res)
    v = n / busy
    return {"value": round(v, 1), "unit": "scans/s", "cores": nproc, "kind": "port", "cpu": cpu_model(),
            "sample": f"{nproc} processes x the oracle IP+FA-feature path, {n} scans in all, slowest process "
                      f"{busy:.1f} s busy ({wall:.1f} s wall incl. start-up)",
            **host_share(v, nproc)}


def pool_map(fn, jobs: list, nproc: int) -> list:
    """multiprocessing map over `nproc` spawned CPU workers, closed and joined (a `with Pool` exit
    terminates its workers with SIGTERM, which a profiler's signal handler logs as an abort)."""
    import multiprocessing as mp
    pool = mp.get_context("spawn").Pool(nproc)
    try:
        res = pool.map(fn, jobs)
    finally:
        pool.close()
        pool.join()
    return res


def host_share(value: float, nproc: int) -> dict:
    """Why the all-core baselines stop at 16 processes, and the whole host's figure next to it."""
    ncpu = os.cpu_count() or nproc
    return {"cores_cap_reason": "16 = the host-CPU share the GPU pool grants one MI355X job (OMP_NUM_THREADS / "
                                "MAX_JOBS are 16 there; more workers than the share would be throttled); on an "
                                "8-GPU node that is also about one GPU's share of the host",
            "host_cpus": ncpu,
            "full_host_extrapolated": round(value / nproc * ncpu, 1),
            "full_host_note": f"linear extrapolation of the per-process rate to all {ncpu} host CPUs "
                              "(an upper bound: SMT siblings and memory bandwidth are shared)"}


def cpu_stage_times(budget_s: float, frames: int = 40) -> dict:
    """BASELINE.md §2 per-stage CPU times of the whole reference pipeline on one VLP-16 drive
    through the oracle chain (oracle_py.OracleMapping, MapOptimization in the lm_applied mode):
    t_IP (ImageProjection), t_FA (feature stage + scan-to-scan LM + integrate + last clouds), t_MO
    (OdometryToTransform .. saveKeyFramesAndFactor incl. the local map); frames after the second
    (the first scan sends no AssociationOut, the second meets an empty map). Sequential scans/s =
    1 / (t_IP + t_FA + t_MO), pipelined (one thread per node, as the reference runs) = 1 / max."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py
    from llsr import _abi, synth
    cfg = _abi.config_for("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    om = oracle_py.OracleMapping(cfg, _abi.LLSR_MODE_LM_APPLIED)
    odo_process = om.odo.process
    t_odo = [0.0]

    def timed_odo(x):
        t1 = time.perf_counter()
        r = odo_process(x)
        t_odo[0] = time.perf_counter() - t1
        return r

    om.odo.process = timed_odo
    ip = fa = mo = 0.0
    n, spent = 0, 0.0
    for k in range(frames):
        scan = synth.make_scan(1 + k, "vlp16", motion=True)
        t1 = time.perf_counter()
        om.process(scan)
        tot = time.perf_counter() - t1
        if k < 2:
            continue
        t_ip = om.odo.ora.stage_ms()[0] * 1e-3
        ip += t_ip
        fa += t_odo[0] - t_ip
        mo += tot - t_odo[0]
        n += 1
        spent += tot
        if spent >= budget_s and n >= 3:
            break
    ip, fa, mo = ip / n * 1e3, fa / n * 1e3, mo / n * 1e3
    return {"per_stage_ms": {"IP": round(ip, 3), "FA": round(fa, 3), "MO_lm_applied": round(mo, 3)},
            "sequential_scans_per_s": round(1e3 / (ip + fa + mo), 2),
            "pipelined_scans_per_s": round(1e3 / max(ip, fa, mo), 2),
            "cores": 1, "cpu": cpu_model(), "mo_mode": "lm_applied",
            "sample": f"frames 3..{n + 2} of one VLP-16 drive through oracle_py.OracleMapping (C++ restatement, "
                      "1 thread per stage)"}


def same_build(record: dict) -> bool:
    """A PMC record under profiles/ counts only for the build it measured (llsr_build_id, a hash
    of the kernel sources): bytes measured on other kernels would be stale evidence."""
    from llsr import build_id
    return record.get("build_id") == build_id()


def lm_traffic(kernel: str, problems: int, leg: str | None = None):
    """PMC-measured HBM bytes per launch of an LM kernel (scripts/pmc_lm.sh, committed as
    profiles/traffic_lm_latest.json; records keyed "kernel" or "kernel@leg"), or None when it was
    measured at another batch size."""
    f = os.environ.get("LLSR_TRAFFIC_LM_JSON", os.path.join(REPO, "profiles", "traffic_lm_latest.json"))
    if not os.path.exists(f):
        return None
    tj = json.load(open(f))
    if not same_build(tj):
        return None
    ks = tj.get("kernels", {})
    rec = ks.get(f"{kernel}@{leg}") if leg else None
    rec = rec or ks.get(kernel)
    if rec and leg and rec.get("leg_key", leg) != leg:
        return None
    return rec["hbm_bytes_per_launch"] if rec and rec.get("problems") == problems else None


def s2m_bytes_per_iteration(Qc: int, Qs: int, blocks: int) -> float:
    """query 16 B + 5 neighbours x 16 B per query, 29 partial words per block."""
    return 96.0 * (Qc + Qs) + 116.0 * blocks


def _s2m_check_worker(args):
    """Oracle poses of a chunk of scan-to-map problems (the parity check of every problem of a
    step, spread over the host cores): [(problem, pose)]."""
    fixture, mode_name, items = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py
    from llsr import _abi, default_config
    cfg = default_config("vlp16")
    cfg.mode = {"lm_applied": _abi.LLSR_MODE_LM_APPLIED, "faithful": _abi.LLSR_MODE_FAITHFUL}[mode_name]
    z = np.load(os.path.join(REPO, "tests", "golden", fixture))
    knn = "kdtree" if oracle_py.ref_lib() is not None else "grid"
    return [(p, oracle_py.scan2map(cfg, z[f"q{q}_corner"], z[f"q{q}_surf"], z["corner_map"], z["surf_map"], pose,
                                   knn=knn)["pose"]) for p, q, pose in items]


def scan2map_leg(dev, mode_name: str, P: int, steps: int, warmup: int, dist, run_cpu: bool,
                 cpu_seconds: float, fixture: str = "mo_map_vlp16.npz") -> dict:
    """Config 3: P independent scan-to-map problems per step; each problem carries its own copy of
    the local map (its kd-tree/grid is rebuilt every step, as MO rebuilds it every scan,
    MO:1575-1576), one of the fixture's query scans and its own seeded start pose."""
    import torch
    from llsr import Pipeline, _abi, default_config
    z = np.load(os.path.join(REPO, "tests", "golden", fixture))
    nq = int(z["n_queries"])
    mode = {"lm_applied": _abi.LLSR_MODE_LM_APPLIED, "faithful": _abi.LLSR_MODE_FAITHFUL}[mode_name]
    cfg = default_config("vlp16")
    cfg.mode = mode
    cm, sm = z["corner_map"], z["surf_map"]
    rng = np.random.default_rng(99)
    probs = []
    for p in range(P):
        q = p % nq
        pose = z[f"q{q}_true"] + np.concatenate([rng.uniform(-0.05, 0.05, 3), rng.uniform(-0.2, 0.2, 3)])
        probs.append((z[f"q{q}_corner"], z[f"q{q}_surf"], cm, sm, pose.astype(np.float32), q))

    def pack(k):
        arrs = [pr[k] for pr in probs]
        off = np.zeros(P + 1, np.int64)
        off[1:] = np.cumsum([len(a) for a in arrs])
        return torch.from_numpy(np.concatenate(arrs)).to(dev), torch.from_numpy(off).to(dev)

    (cq, cqo), (sq, sqo), (dcm, cmo), (dsm, smo) = (pack(k) for k in range(4))
    pose0 = torch.from_numpy(np.stack([pr[4] for pr in probs])).to(dev)
    pose = pose0.clone()
    rep = torch.zeros((P, ctypes_sizeof_report() // 4), dtype=torch.float32, device=dev)
    pipe = Pipeline(cfg, device=dev)
    Qc = max(len(pr[0]) for pr in probs)
    Qs = max(len(pr[1]) for pr in probs)
    pipe.scan2map_reserve(P, len(cm), len(sm), Qc, Qs)
    ptrs = dict(corner_q=cq.data_ptr(), corner_q_off=cqo.data_ptr(), surf_q=sq.data_ptr(),
                surf_q_off=sqo.data_ptr(), corner_map=dcm.data_ptr(), corner_map_off=cmo.data_ptr(),
                surf_map=dsm.data_ptr(), surf_map_off=smo.data_ptr(), pose=pose.data_ptr(),
                report=rep.data_ptr())
    stream = torch.cuda.Stream(dev)  # the pose reset and the batch on one (non-default) stream

    def step():
        with torch.cuda.stream(stream):
            pose.copy_(pose0)  # every step solves the same P problems from their start poses
            pipe.scan2map_batch(ptrs, P, stream.cuda_stream)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    pipe.set_profiling(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    st = pipe.scan2map_stats()
    pipe.set_profiling(False)
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    world = dist.get_world_size() if dist else 1
    from llsr import _abi as abi_
    raw = rep.cpu().numpy().tobytes()
    n = ctypes_sizeof_report()
    reps = [abi_.LmReport.from_buffer_copy(raw[p * n:(p + 1) * n]) for p in range(P)]
    iters = np.array([r.iterations for r in reps], np.float64)
    poses = pose.cpu().numpy()
    blocks = (Qc + 255) // 256 + (Qs + 255) // 256
    lm_bytes = sum(r.iterations * s2m_bytes_per_iteration(len(pr[0]), len(pr[1]), blocks)
                   for r, pr in zip(reps, probs))
    per_launch_ms = st["iterate_ms"] / max(1, st["iteration_launches"])
    launches_per_batch = st["iteration_launches"] / max(1, st["batches"])
    achieved = lm_bytes / (st["iterate_ms"] / max(1, st["batches"]) * 1e-3) / 1e9
    tr = lm_traffic("k_s2m_iter", P)
    out = {
        "workload": "configs[2]: scan-to-map LM (corner/surf kNN-5 correspondences + 6x6 normal "
                    f"equations + solve) against a {len(cm) + len(sm)}-point local map, mode {mode_name}",
        "value": round(P * steps * world / el, 1), "unit": "scan-to-map problems/s",
        "problems_per_gpu_per_step": P, "steps": steps, "ms_per_step": round(el / steps * 1e3, 3),
        "map_points": {"corner": len(cm), "surf": len(sm)},
        "queries_per_problem": {"corner": float(np.mean([len(pr[0]) for pr in probs])),
                                "surf": float(np.mean([len(pr[1]) for pr in probs]))},
        "iterations_mean": float(iters.mean()), "iterations_max": int(iters.max()),
        "converged_frac": float(np.mean([r.converged for r in reps])),
        "grid_build_ms_per_step": round(st["grid_ms"] / max(1, st["batches"]), 4),
        "iterate_ms_per_step": round(st["iterate_ms"] / max(1, st["batches"]), 4),
        "k_s2m_iter_launches_per_step": launches_per_batch,
        "roofline": {"bound": "hbm", "kernel": "k_s2m_iter", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": tr, "algorithmic_bytes_per_step": lm_bytes,
                     "traffic_per_step": tr * launches_per_batch if tr is not None else None,
                     "traffic_over_algorithmic": round(tr * launches_per_batch / lm_bytes, 2) if tr is not None else None,
                     "algorithmic_bytes_per_launch": lm_bytes / max(1, launches_per_batch),
                     "avg_launch_ms": round(per_launch_ms, 4),
                     "note": "bytes = SURVEY 8(d) B_lm per iteration; iterate window includes the host's "
                             "convergence polls (every 4 launches); traffic = PMC HBM bytes per launch "
                             "(the kNN-5 cell walks and the maps beyond the XCD L2s)"},
    }
    if run_cpu:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle_py
        knn = "kdtree" if oracle_py.ref_lib() is not None else "grid"
        # CPU baseline: the restatement on one core, problem after problem, for ~cpu_seconds
        t_cpu, n_cpu = 0.0, 0
        while t_cpu < cpu_seconds and n_cpu < 10000:
            o = oracle_py.scan2map(cfg, *probs[n_cpu % P][:5], knn=knn)
            t_cpu += o["ms"] * 1e-3
            n_cpu += 1
        # parity: every problem of the step against the oracle, spread over the host cores
        nproc = min(16, os.cpu_count() or 1, P)
        items = [(p, probs[p][5], probs[p][4]) for p in range(P)]
        res = pool_map(_s2m_check_worker, [(fixture, mode_name, items[k::nproc]) for k in range(nproc)], nproc)
        deltas = [float(np.abs(poses[p] - po).max()) for chunk in res for p, po in chunk]
        out["pose_delta_max"] = max(deltas)
        out["pose_delta_problems"] = len(deltas)
        out["bit_exact_problems"] = int(sum(d == 0.0 for d in deltas))
        out["cpu_baseline"] = {
            "value": round(n_cpu / t_cpu, 2), "unit": "scan-to-map problems/s", "cores": 1, "kind": "port",
            "sample": f"{n_cpu} problems of this batch through the C++ MO restatement ({mode_name}, kNN = "
                      f"{'the reference nanoflann kd-tree, oracle/_ref' if knn == 'kdtree' else 'grid restatement'}"
                      f", tree build included), 1 thread, {t_cpu:.1f} s"}
        out["speedup_vs_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    pipe.close()
    return out


def scan2map_allreduce_leg(dev, P: int, steps: int, warmup: int, dist, check: bool) -> dict:
    """configs[4]: B = P scans per step, every scan's scan-to-map correspondences split over all
    ranks (llsr_scan2map_shard_*), ONE RCCL all-reduce of the [P][32] int64 normal equations per
    LM iteration (llsr.dist.sharded_scan2map); every rank solves the same 6x6 systems. The total
    work is fixed as N grows (strong scaling of one batch); at N = 1 the all-reduce still runs
    through RCCL on a one-rank group (an in-place identity), so allreduce_us is RCCL's latency."""
    import torch
    from llsr import Pipeline, _abi, default_config
    from llsr.dist import HipShardEngine, allreduce_latency_us, max_over_ranks, sharded_scan2map
    z = np.load(os.path.join(REPO, "tests", "golden", "mo_map_vlp16.npz"))
    nq = int(z["n_queries"])
    cfg = default_config("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    rng = np.random.default_rng(7)
    probs = []
    for p in range(P):
        q = p % nq
        pose = z[f"q{q}_true"] + np.concatenate([rng.uniform(-0.05, 0.05, 3), rng.uniform(-0.2, 0.2, 3)])
        probs.append((z[f"q{q}_corner"], z[f"q{q}_surf"], z["corner_map"], z["surf_map"], pose.astype(np.float32)))

    def pack(k):
        arrs = [pr[k] for pr in probs]
        off = np.zeros(P + 1, np.int64)
        off[1:] = np.cumsum([len(a) for a in arrs])
        return torch.from_numpy(np.concatenate(arrs)).to(dev), torch.from_numpy(off).to(dev)

    (cq, cqo), (sq, sqo), (dcm, cmo), (dsm, smo) = (pack(k) for k in range(4))
    pose0 = torch.from_numpy(np.stack([pr[4] for pr in probs])).to(dev)
    pose = pose0.clone()
    rep = torch.zeros((P, ctypes_sizeof_report() // 4), dtype=torch.float32, device=dev)
    pipe = Pipeline(cfg, device=dev)
    pipe.scan2map_reserve(P, len(z["corner_map"]), len(z["surf_map"]), max(len(pr[0]) for pr in probs),
                          max(len(pr[1]) for pr in probs))
    ptrs = dict(corner_q=cq.data_ptr(), corner_q_off=cqo.data_ptr(), surf_q=sq.data_ptr(),
                surf_q_off=sqo.data_ptr(), corner_map=dcm.data_ptr(), corner_map_off=cmo.data_ptr(),
                surf_map=dsm.data_ptr(), surf_map_off=smo.data_ptr(), pose=pose.data_ptr(),
                report=rep.data_ptr())
    side = torch.cuda.Stream(dev)  # torch's ops, the library's kernels and RCCL on one stream
    ctx = torch.cuda.stream(side)
    ctx.__enter__()
    eng = HipShardEngine(pipe, ptrs, P, side.cuda_stream)
    ne = eng.new_ne(dev)
    iters = []

    def step():
        pose.copy_(pose0)
        # the all-reduce runs through RCCL at every world size (at N = 1: a one-rank group)
        iters.append(sharded_scan2map(eng, ne, cfg.iterCountThres, poll=2, force_collective=True))

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0, dev)
    lat = allreduce_latency_us(ne)
    ctx.__exit__(None, None, None)
    out = {"workload": f"configs[4]: {P} scans per step, each scan's scan-to-map correspondences split over "
                       "all ranks, one all-reduce of the [P][32] int64 normal equations per LM iteration "
                       "(lm_applied, ~100k-point local map)",
           "value": round(P * steps / el, 1), "unit": "scans/s", "scaling": "strong",
           "scans_per_step": P, "steps": steps, "ms_per_step": round(el / steps * 1e3, 3),
           "lm_iterations_per_step": float(np.mean(iters[warmup:] if len(iters) > warmup else iters)),
           "allreduce_bytes": P * 32 * 8, "allreduce_us": round(lat, 2)}
    if check:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle_py
        poses = pose.cpu().numpy()
        out["pose_delta_max"] = max(float(np.abs(poses[p] - oracle_py.scan2map(cfg, *probs[p])["pose"]).max())
                                    for p in range(min(P, nq)))
    pipe.close()
    return out


def odometry_leg(dev, lidar: str, B: int, seqs: int, frames: int, steps: int, warmup: int, dist,
                 check: bool, cpu_seconds: float) -> dict:
    """configs[3] (HDL-64E) / VLP-16: end-to-end odometry of B independent sequences, one scan per
    sequence per step: IP + feature stage + scan-to-scan LM + integrateTransformation + the next
    last clouds, all on the device (llsr_odometry_batch). `seqs` distinct synthetic drives of
    `frames` consecutive scans (0.5 m apart, the sensor moving in 6 DoF: synth.sensor_attitude) are
    tiled over the slots; `frames` covers the warm-up and timed steps, so every measured step is a
    real frame-to-frame transition. The per-kernel times come from a replay of the SAME frames:
    after the timed region every slot is reset and the drive runs again from frame 0, its timed
    frames with HIP events between the kernels, so the roofline describes the timed work."""
    import torch
    from llsr import Pipeline, _abi, default_config, synth
    from llsr.dist import max_over_ranks
    hdl = lidar == "hdl64e"
    cfg = default_config(lidar, 2048 if hdl else None)
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    H, W = cfg.num_vertical_scans, cfg.num_horizontal_scans
    rank = dist.get_rank() if dist else 0
    seq_scans = [[synth.make_scan(1 + 64 * (q + 4 * rank) + k, lidar, motion=True) for k in range(frames)]
                 for q in range(seqs)]
    batches = []
    for k in range(frames):
        scans = [seq_scans[b % seqs][k] for b in range(B)]
        off = np.zeros(B + 1, np.int64)
        off[1:] = np.cumsum([len(a) for a in scans])
        batches.append((torch.from_numpy(np.concatenate(scans)).to(dev), torch.from_numpy(off).to(dev)))
    pipe = Pipeline(cfg, device=dev, max_batch=B, max_points=H * W)
    torch.cuda.synchronize(dev)
    n = 0

    def step():
        nonlocal n
        d_pts, d_off = batches[n % frames]
        pipe.odometry_batch(d_pts.data_ptr(), d_off.data_ptr(), B)
        n += 1

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0, dev)
    world = dist.get_world_size() if dist else 1
    # per-kernel device times (HIP events on the launch stream) of the timed frames: reset, replay
    # the warm-up frames, then the timed frames again with profiling on (the same state, the same
    # work): the IP + feature kernels of llsr_process_batch and the scan-to-scan grid build + LM
    pipe.odometry_reset()
    n = 0
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    pipe.set_profiling(True)
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    kt = pipe.kernel_times()
    st = pipe.scan2scan_stats()
    pipe.set_profiling(False)
    cnt = pipe.batch_counts(B)  # N, S, O, M, sharp, F, L, K of the last batch
    # k_s2s_lm's compulsory HBM bytes per launch: each query (sharp + flat + shadow,
    # 16 B) and each point of the two last clouds' cell-sorted copies (16 B) read once; the
    # per-iteration re-reads stay on chip (LDS / L2) and are not counted, so this is a lower bound
    # that the PMC `traffic` must meet (model <= traffic)
    reps = [pipe.odometry_fetch(b)["lm"] for b in range(0, B, max(1, B // 64))]
    q_mean = float(np.mean(cnt[:, 4] + cnt[:, 5] + 160))
    it_mean = float(np.mean([r["surf_iterations"] + r["corner_iterations"] for r in reps]))
    surf_it = [r["surf_iterations"] for r in reps if not r["skipped"]]
    last_mean = float(np.mean(cnt[:, 3] + cnt[:, 6] + 160))  # M + L + shadow: the next frame's last clouds
    lm_bytes = B * 16.0 * (q_mean + last_mean)
    lm_ms = st["lm_ms"] / max(1, st["batches"])
    N = float(cnt[:, 0].sum())
    proj_ms = kt["k_project"] + kt["k_gather_column"]
    bpc_proj = 20 * N + (24 + 1) * float(H * W * B)
    def roof(kname, nbytes, ms, note):
        a = nbytes / (ms * 1e-3) / 1e9
        return {"bound": "hbm", "kernel": kname, "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(a / HBM_PEAK_GBS, 4), "traffic": None, "algorithmic_bytes_per_launch": nbytes,
                "avg_launch_ms": round(ms, 4), "note": note}
    s0 = pipe.odometry_fetch(0)
    out = {"workload": f"{'configs[3]: HDL-64E 64x2048' if hdl else 'VLP-16 1800x16'} end-to-end odometry: "
                       "projection + segmentation + features + scan-to-scan LM + transformSum + last clouds, "
                       f"{B} sequences per GPU, one scan each per step",
           "value": round(B * steps * world / el, 1), "unit": "scans/s", "scaling": "weak",
           "sequences_per_gpu": B, "steps": steps, "ms_per_step": round(el / steps * 1e3, 3),
           "slot0_frames": s0["frames"], "slot0_lm_iterations": [s0["lm"]["surf_iterations"], s0["lm"]["corner_iterations"]],
           "roofline": {**roof("k_s2s_lm", lm_bytes, lm_ms,
                                "dominant kernel of the leg; compulsory bytes = 16 B per query + 16 B per "
                                "last-cloud point, each read once per launch (iterations re-read on chip); "
                                "latency-bound (one workgroup per scan, ordered sums); traffic = PMC HBM "
                                "bytes per launch"),
                         "traffic": lm_traffic("k_s2s_lm", B, "odometry " + lidar)},
           "roofline_projection": roof("k_project" if not hdl else "k_project+k_gather_column", bpc_proj, proj_ms,
                                       "SURVEY 8(d) B_pc projection part 20 N + 24 HW (+ 1 HW ground) "
                                       "over the projection kernels"),
           "kernels_ms_per_step": {**{k: round(v, 4) for k, v in kt.items()},
                                   "s2s_grid_build": round(st["grid_ms"] / max(1, st["batches"]), 4),
                                   "k_s2s_lm": round(lm_ms, 4)},
           "lm_iterations_mean": it_mean, "lm_queries_mean": q_mean,
           "surf_iterations_mean": round(float(np.mean(surf_it)), 2) if surf_it else None,
           "surf_iterations_max": int(max(surf_it)) if surf_it else None}
    if check:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle_py
        # slot 0 replays sequence 0 frame (i % frames) for i = 0 .. n-1: the oracle does the same,
        # in the reference's (PCL) VoxelGrid order like the device, and once more in ring order to
        # show what the summation order alone moves (the less-flat cloud becomes the next scan's
        # laserCloudSurfLast, FA:2660-2712)
        od = oracle_py.OracleOdometry(cfg)
        odi = oracle_py.OracleOdometry(cfg, pcl_voxel_order=False)
        t_cpu, dord = 0.0, 0.0
        for i in range(n):
            t1 = time.perf_counter()
            o = od.process(seq_scans[0][i % frames])
            t_cpu += time.perf_counter() - t1
            oi = odi.process(seq_scans[0][i % frames])
            dord = max(dord, float(np.abs(o["transform_sum"] - oi["transform_sum"]).max()))
        out["pose_delta_max"] = float(max(np.abs(s0["transform_cur"] - o["transform_cur"]).max(),
                                          np.abs(s0["transform_sum"] - o["transform_sum"]).max()))
        out["voxel_order"] = "pcl (std::sort, as the reference)"
        out["input_order_transform_sum_delta_max"] = dord
        # CPU baseline: the same restatement, one core, continuing the sequence for ~cpu_seconds
        k = n
        while t_cpu < cpu_seconds and k < n + 1000:
            t1 = time.perf_counter()
            od.process(seq_scans[0][k % frames])
            t_cpu += time.perf_counter() - t1
            k += 1
        out["cpu_baseline"] = {"value": round(k / t_cpu, 2), "unit": "scans/s", "cores": 1, "kind": "port",
                               "sample": f"{k} scans of sequence 0 through the oracle (IP + features + "
                                         f"scan-to-scan LM + integrate + TransformToEnd), 1 thread, {t_cpu:.1f} s"}
        out["speedup_vs_cpu"] = round(out["value"] / world / out["cpu_baseline"]["value"], 1)
    pipe.close()
    return out


def _mapping_cpu_worker(args):
    """One CPU process of the mapping leg's multi-core baseline: the oracle chain over one sequence,
    timing frames >= `skip` only (the same frame indices the device leg times)."""
    seed0, frames, skip, mo_mode, budget = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py
    from llsr import _abi, synth
    cfg = _abi.config_for("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    om = oracle_py.OracleMapping(cfg, mo_mode)
    n, t = 0, 0.0
    for k in range(frames):
        scan = synth.make_scan(seed0 + k, "vlp16", motion=True)
        t1 = time.perf_counter()
        om.process(scan)
        if k >= skip:
            t += time.perf_counter() - t1
            n += 1
        if t > budget:
            break
    return n, t


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def mapping_leg(dev, B: int, seqs: int, warmup: int, steps: int, dist, check: bool, cpu_seconds: float,
                mo_mode_name: str = "lm_applied") -> dict:
    """The mapping chain (llsr_mapping_batch): B independent VLP-16 drives, one scan each per step,
    through ImageProjection + features + scan-to-scan LM + OdometryToTransform +
    transformAssociateToMap + extractSurroundingKeyFrames + downsampleCurrentScan + scan-to-map LM +
    transformUpdate + keyframe, all slots batched on the device. `seqs` distinct drives (0.5 m
    between scans) are tiled over the slots; the timed steps are frames warmup .. warmup+steps-1
    of every drive (the local map keeps growing: every frame is a keyframe, MO:1629)."""
    import torch
    from llsr import Pipeline, _abi, default_config, synth
    from llsr.dist import max_over_ranks
    mo_mode = {"lm_applied": _abi.LLSR_MODE_LM_APPLIED, "faithful": _abi.LLSR_MODE_FAITHFUL}[mo_mode_name]
    cfg = default_config("vlp16")
    cfg.mode = _abi.LLSR_MODE_LM_APPLIED
    H, W = cfg.num_vertical_scans, cfg.num_horizontal_scans
    rank = dist.get_rank() if dist else 0
    frames = warmup + steps
    seeds = [1 + 64 * (q + 4 * rank) for q in range(seqs)]
    seq_scans = [[synth.make_scan(s0 + k, "vlp16", motion=True) for k in range(frames)] for s0 in seeds]
    batches = []
    for k in range(frames):
        scans = [seq_scans[b % seqs][k] for b in range(B)]
        off = np.zeros(B + 1, np.int64)
        off[1:] = np.cumsum([len(a) for a in scans])
        batches.append((torch.from_numpy(np.concatenate(scans)).to(dev), torch.from_numpy(off).to(dev)))
    pipe = Pipeline(cfg, device=dev, max_batch=B, max_points=H * W)
    pipe.mapping_init(mo_mode)
    torch.cuda.synchronize(dev)
    for k in range(warmup):
        pipe.mapping_batch(batches[k][0].data_ptr(), batches[k][1].data_ptr(), B)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(warmup, frames):
        pipe.mapping_batch(batches[k][0].data_ptr(), batches[k][1].data_ptr(), B)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0, dev)
    world = dist.get_world_size() if dist else 1
    s0 = pipe.mapping_fetch(0)
    out = {"workload": f"VLP-16 mapping chain: IP + features + scan-to-scan LM + MapOptimization::run "
                       f"(local map, downsample, scan-to-map LM mode {mo_mode_name}, keyframes), {B} drives per "
                       f"GPU, frames {warmup}..{frames - 1} of each (every frame a keyframe)",
           "value": round(B * steps * world / el, 1), "unit": "scans/s", "scaling": "weak", "steps": steps,
           "drives_per_gpu": B, "ms_per_step": round(el / steps * 1e3, 3),
           "slot0": {"keyframes": s0["keyframes"], "lm_iterations": s0["lm"]["iterations"],
                     "corner_map_ds": s0["map"]["n_corner_ds"], "surf_map_ds": s0["map"]["n_surf_ds"],
                     "corner_q": s0["n_corner_q"], "surf_q": s0["n_surf_q"]}}
    if check:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle_py
        om = oracle_py.OracleMapping(cfg, mo_mode)
        t_cpu = 0.0
        for k in range(frames):
            t1 = time.perf_counter()
            o = om.process(seq_scans[0][k])
            if k >= warmup:
                t_cpu += time.perf_counter() - t1
        out["bit_exact_slot0"] = bool(all(np.array_equal(s0[key], o[key]) for key in
                                          ("transform_sum", "transform_tobe_mapped", "transform_aft_mapped")))
        n1 = steps
        out["cpu_baseline"] = {"value": round(n1 / t_cpu, 2), "unit": "scans/s", "cores": 1, "kind": "port",
                               "cpu": cpu_model(),
                               "sample": f"frames {warmup}..{frames - 1} of drive 0 through the oracle chain "
                                         f"(oracle_py.OracleMapping), 1 thread, {t_cpu:.1f} s"}
        # every host core the box grants this job (16 on the GPU pool): one drive per process
        nproc = min(16, os.cpu_count() or 1)
        jobs = [(1 + 64 * (q + 4 * rank) + 256 * (q // seqs), frames, warmup, mo_mode, cpu_seconds)
                for q in range(nproc)]
        t1 = time.perf_counter()
        res = pool_map(_mapping_cpu_worker, jobs, nproc)
        wall = time.perf_counter() - t1
        nf = sum(r[0] for r in res)
        busy = max(r[1] for r in res)
        out["cpu_baseline_all_cores"] = {
            "value": round(nf / busy, 2), "unit": "scans/s", "cores": nproc, "kind": "port", "cpu": cpu_model(),
            "sample": f"{nproc} processes, one drive each, frames {warmup}..{frames - 1} timed ({nf} frames, "
                      f"slowest process {busy:.1f} s busy, {wall:.1f} s wall incl. start-up and untimed frames)",
            **host_share(nf / busy, nproc)}
        out["speedup_vs_cpu"] = round(out["value"] / world / out["cpu_baseline"]["value"], 1)
        out["speedup_vs_cpu_all_cores"] = round(out["value"] / world / out["cpu_baseline_all_cores"]["value"], 1)
    pipe.close()
    return out


def local_map_leg(dev, K: int, steps: int, warmup: int, dist, check: bool, cpu_seconds: float) -> dict:
    """MapOptimization local map (llsr_map_extract, MO:1096-1232): a store of K synthetic keyframes
    (VLP-16-sized clouds: 200 corner, 6000 surf, 1500 outlier points) along an out-and-back path;
    one step = extractSurroundingKeyFrames at the next robot position (radius 50 m, key-pose
    VoxelGrid 1.0, list update, transform, VoxelGrid 0.2 / 0.4), synchronous like the reference.
    Each rank owns its map (independent sequences: weak scaling, no collective)."""
    import torch
    from llsr import LocalMap, synth
    from llsr.dist import max_over_ranks
    rank = dist.get_rank() if dist else 0
    frames = synth.make_keyframes(K, seed=17 + rank, corner=200, surf=6000, outlier=1500)
    m = LocalMap(dev)
    for pose, c, s, o in frames:
        m.add_keyframe(pose, torch.from_numpy(c).to(dev), torch.from_numpy(s).to(dev), torch.from_numpy(o).to(dev))
    positions = [frames[(7 * i) % K][0][:3] + np.float32(0.25) for i in range(warmup + steps)]
    reps = []
    for i in range(warmup):
        m.extract(positions[i])
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        gc, gs, rep = m.extract(positions[i])
        reps.append(rep)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0, dev)
    world = dist.get_world_size() if dist else 1
    pts = float(np.mean([r["n_corner_map"] + r["n_surf_map"] for r in reps]))
    out = {"workload": f"extractSurroundingKeyFrames over {K} stored keyframes (200/6000/1500 pts), "
                       "radius 50 m, VoxelGrid 0.2 / 0.4 of the assembled local map, one extract per step",
           "value": round(steps * world / el, 1), "unit": "extracts/s", "scaling": "weak", "steps": steps,
           "ms_per_extract": round(el / steps * 1e3, 3),
           "map_points_per_extract": round(pts), "keyframes_per_extract": float(np.mean([r["n_keyframes"] for r in reps])),
           "map_points_per_s": round(pts * steps * world / el, 1),
           "ds_points_per_extract": round(float(np.mean([r["n_corner_ds"] + r["n_surf_ds"] for r in reps])))}
    if check:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle_py
        # the device sums each voxel in std::sort's order (PCL), as the PCL-order restatement does
        op = oracle_py.OracleMap(stable=False)
        for pose, c, s, o in frames:
            op.add_keyframe(pose, c, s, o)
        for i, p in enumerate(positions):
            rc, rs, _, _ = op.extract(p)
        out["bit_exact_last_extract"] = bool(
            np.array_equal(gc.cpu().numpy().view(np.uint32), rc.view(np.uint32))
            and np.array_equal(gs.cpu().numpy().view(np.uint32), rs.view(np.uint32)))
        # CPU baseline: the same restatement, one core, bounded (continues the path)
        t_cpu, n_cpu, i = 0.0, 0, 0
        while t_cpu < cpu_seconds and n_cpu < 200:
            t1 = time.perf_counter()
            op.extract(positions[i % len(positions)])
            t_cpu += time.perf_counter() - t1
            n_cpu += 1
            i += 1
        out["cpu_baseline"] = {"value": round(n_cpu / t_cpu, 2), "unit": "extracts/s", "cores": 1, "kind": "port",
                               "sample": f"{n_cpu} extracts on the same map and path through oracle_map_extract "
                                         f"(std::sort VoxelGrid as PCL), 1 thread, {t_cpu:.1f} s"}
        out["speedup_vs_cpu"] = round(out["value"] / world / out["cpu_baseline"]["value"], 1)
    m.close()
    return out


def pc2_decode_leg(dev, pts: np.ndarray, off: np.ndarray, steps: int, dist) -> dict:
    """sensor_msgs/PointCloud2 -> PointXYZI (pcl::fromROSMsg, IP:196; llsr_decode_pointcloud2) of the
    bench's own B scans encoded in the velodyne_pointcloud layout (x, y, z, intensity, ring, time;
    point_step 32), message bytes resident in HBM. One step = one decode call of the whole batch
    (host table upload + k_decode_pc2 + sync). Algorithmic bytes: 32 read + 16 written per point."""
    import ctypes as C
    import torch
    import llsr
    from llsr import _abi
    from llsr.dist import max_over_ranks
    B = len(off) - 1
    n = int(off[-1])
    rec = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("pad", "<f4"), ("intensity", "<f4"),
                             ("ring", "<u2"), ("pad2", "<u2"), ("time", "<f4"), ("pad3", "<f4")])
    for a, name in enumerate(("x", "y", "z", "intensity")):
        rec[name] = pts[:, a]
    data = torch.from_numpy(rec.view(np.uint8).reshape(-1)).to(dev)
    lay = llsr.pc2_layout([("x", 0, 7, 1), ("y", 4, 7, 1), ("z", 8, 7, 1), ("intensity", 16, 7, 1),
                           ("ring", 20, 4, 1), ("time", 24, 7, 1)], 32)
    msgs = (_abi.Pc2Msg * B)()
    for b in range(B):
        w = int(off[b + 1] - off[b])
        msgs[b].data_offset, msgs[b].width, msgs[b].height, msgs[b].row_step = int(off[b]) * 32, w, 1, 32 * w
    out = torch.empty((n, 4), dtype=torch.float32, device=dev)
    hoff = np.zeros(B + 1, np.int64)
    d_off = torch.empty(B + 1, dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)

    def step():
        rc = llsr.lib().llsr_decode_pointcloud2(C.byref(lay), C.c_void_p(data.data_ptr()), msgs, B,
                                                C.c_void_p(out.data_ptr()), hoff.ctypes.data,
                                                C.c_void_p(d_off.data_ptr()), C.c_void_p(stream.cuda_stream))
        assert rc == 0, rc

    step()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if dist:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0, dev)
    world = dist.get_world_size() if dist else 1
    exact = bool(np.array_equal(out.cpu().numpy().view(np.uint32), np.ascontiguousarray(pts, np.float32).view(np.uint32)))
    gbs = 48.0 * n / (el / steps) / 1e9
    return {"workload": f"PointCloud2 decode of {B} VLP-16 messages per GPU (velodyne layout, point_step 32)",
            "value": round(B * steps * world / el, 1), "unit": "messages/s", "scaling": "weak",
            "ms_per_call": round(el / steps * 1e3, 4), "points_per_call": n,
            "algorithmic_GBs_incl_host_sync": round(gbs, 1), "bit_exact": exact}


def ctypes_sizeof_report() -> int:
    import ctypes
    from llsr import _abi
    return ctypes.sizeof(_abi.LmReport)


def launcher_cmd(argv: list, gpus: int, port: int) -> list:
    """The torchrun command that runs this script on `gpus` ranks (one process per GPU, RCCL)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=2048, help="scans per GPU per step")
    ap.add_argument("--distinct", type=int, default=16, help="distinct synthetic scans per rank")
    ap.add_argument("--streams", type=int, default=3,
                    help="handles/HIP streams used round-robin, so consecutive batches overlap")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--prof-batches", type=int, default=3,
                    help="single-stream batches timed per kernel for the roofline (after the timed region)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--s2m-problems", type=int, default=256, help="scan-to-map problems per GPU per step")
    ap.add_argument("--s2m-steps", type=int, default=5)
    ap.add_argument("--s2m-modes", default="lm_applied,faithful", help="comma list; empty = skip the leg")
    ap.add_argument("--s2m-fixture", default="mo_map_vlp16.npz", help="tests/golden map fixture of the leg")
    ap.add_argument("--odo", default="hdl64e:512,vlp16:1024",
                    help="odometry legs lidar:sequences_per_gpu, comma list (empty = skip)")
    ap.add_argument("--map-keyframes", type=int, default=200,
                    help="local-map leg: keyframes in the store (0 = skip)")
    ap.add_argument("--pc2", type=int, default=1, help="PointCloud2 decode leg (0 = skip)")
    ap.add_argument("--mapping", default="256:8:8",
                    help="mapping-chain leg drives_per_gpu:warmup_frames:timed_frames (empty = skip)")
    ap.add_argument("--voxel-order", choices=("pcl", "input"), default="pcl",
                    help="less-flat VoxelGrid summation order: pcl = std::sort's (the reference), input = ring order")
    ap.add_argument("--allreduce-scans", type=int, default=8,
                    help="configs[4] leg: scans per step split over all ranks (0 = skip)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # not started by torchrun: launch one rank per GPU as a child process (nothing here has
        # touched the GPU yet) and exit with its status
        sys.exit(subprocess.call(launcher_cmd(sys.argv[1:], args.gpus, free_port())))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    rccl1 = None  # world 1: a one-rank RCCL group for the configs[4] leg's per-iteration all-reduce
    if world == 1 and args.allreduce_scans > 0:
        import torch.distributed as rccl1
        rccl1.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                                 device_id=torch.device("cuda", dev))

    from llsr import Pipeline, build_id, default_config, synth
    cfg = default_config("vlp16")
    H, W = cfg.num_vertical_scans, cfg.num_horizontal_scans
    B = args.batch
    pts, off = synth.make_batch(B, "vlp16", distinct=args.distinct, seed0=1 + 1000 * rank)
    d_pts = torch.from_numpy(pts).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    nS = max(1, args.streams)
    pipes = [Pipeline(cfg, device=dev, max_batch=B, max_points=int(np.diff(off).max())) for _ in range(nS)]
    for p_ in pipes:
        p_.set_voxel_order(VOXEL_ORDERS[args.voxel_order])
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nS - 1)]
    pipe = pipes[0]
    torch.cuda.synchronize(dev)

    def step(k):
        pipes[k % nS].process_batch(d_pts.data_ptr(), d_off.data_ptr(), B, streams[k % nS].cuda_stream)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    # Per-kernel device times for the roofline: a separate pass of `prof_batches` batches on ONE
    # stream (HIP events recorded on the launch stream between the kernels of each batch), so the
    # other streams' concurrent kernels do not stretch the intervals. Same data, same kernels.
    pipe.set_profiling(True)
    for _ in range(args.prof_batches):
        pipe.process_batch(d_pts.data_ptr(), d_off.data_ptr(), B, streams[0].cuda_stream)
    ktimes = pipe.kernel_times()  # ms per batch
    pipe.set_profiling(False)
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # per-scan counts for the algorithmic-byte model, and a parity spot check of slot 0
    cnt = pipe.batch_counts(B)  # N, S, O, M, sharp, F, L, K
    finite = np.isfinite(pts[:, 0]) & np.isfinite(pts[:, 1]) & np.isfinite(pts[:, 2])
    csum = {"Nr": float(np.diff(off).sum()), "N": float(cnt[:, 0].sum()), "S": float(cnt[:, 1].sum()),
            "M": float(cnt[:, 3].sum()), "F": float(cnt[:, 5].sum()), "L": float(cnt[:, 6].sum()),
            "K": float(cnt[:, 7].sum())}
    assert int(finite.sum()) == int(csum["N"])
    r0 = pipe.fetch(0)
    csum["R"] = float(r0["ransac_iterations"])
    csum["M2"] = float((cnt[:, 3].astype(np.float64) ** 2).sum())  # DBSCAN pair count
    HWB = float(H * W * B)
    per = {k: kernel_bytes(k, csum, HWB) for k in ktimes}
    fused = H <= 16 and H * W <= 32768
    if fused:  # fused projection kernel (H*W fits LDS): one launch does both
        per["k_project"] += per["k_gather_column"]
        per["k_gather_column"] = 0.0
    # SURVEY.md 8(d) B_pc: 20 N + 24 HW for the projection (each input point read once and its index
    # scattered; range, XYZI and cell->point index written per cell) + 29 S for the curvature; the
    # fused kernel's other output (the ground byte per cell) is credited too; the per-cell XYZI keeps
    # the raw intensity in w (fullCloud's row + col / 1e4 is derived where needed).
    # Re-reads (the winners' points gathered again) are not algorithmic: they show up in `traffic`.
    bpc_proj = 20 * csum["N"] + (24 + 1) * HWB
    bpc_curv = 29 * csum["S"]
    # the feature selection is k_select_ring + k_vox_pcl (the PCL-order VoxelGrid, split off so its
    # sort runs at a higher occupancy): one stage for the dominance test and its roofline
    sel_ms = ktimes["k_select_ring"] + ktimes.get("k_vox_pcl", 0.0)
    dom = max((k for k in ktimes if k not in ("init", "k_vox_pcl")),
              key=lambda k: sel_ms if k == "k_select_ring" else ktimes[k])
    total_scans = B * args.steps * world
    value = total_scans / el
    parity = None
    if rank == 0 and not args.no_cpu:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_py
        from _compare import compare
        # slot 0 of handle 0 has seen every nS-th batch of the same cloud: replay that history
        ora = oracle_py.Oracle(cfg, pcl_voxel_order=args.voxel_order == "pcl")
        n0 = len(range(0, args.warmup, nS)) + len(range(0, args.steps, nS)) + args.prof_batches
        for _ in range(n0):
            o = ora.process(pts[off[0]:off[1]])
        parity = not compare(r0, o)

    # PMC-measured HBM bytes per launch (scripts/pmc.sh, committed under profiles/), per scan
    # scaled to this batch size; null when no measurement for this kernel exists.
    tfile = os.environ.get("LLSR_TRAFFIC_JSON", os.path.join(REPO, "profiles", "traffic_latest.json"))
    tjson = json.load(open(tfile)) if os.path.exists(tfile) else {}
    if not same_build(tjson):
        tjson = {}

    def traffic_of(kname):
        if kname == "k_project" and fused:
            kname = "k_project_fused"  # the VLP-16 launch's own name in the PMC record
        rec = tjson.get("kernels", {}).get(kname)
        return rec["hbm_bytes"] / tjson["batch"] * B if rec and tjson.get("batch") else None

    def roofline(kname, nbytes=None, ms=None, traffic=None, note=None):
        nbytes = per[kname] if nbytes is None else nbytes
        ms = ktimes[kname] if ms is None else ms
        a = nbytes / (ms * 1e-3) / 1e9
        out = {"bound": "hbm", "kernel": kname, "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(a / HBM_PEAK_GBS, 4), "traffic": traffic_of(kname) if traffic is None else traffic,
               "algorithmic_bytes_per_launch": nbytes, "avg_launch_ms": round(ms, 4)}
        if note:
            out["note"] = note
        return out

    proj_ms = ktimes["k_project"] + (0.0 if fused else ktimes["k_gather_column"])
    tp = traffic_of("k_project")
    roof_proj = roofline("k_project", bpc_proj, proj_ms, note="B_pc projection part: 20 N + 24 HW (+ 1 HW "
                         "ground output); traffic = PMC bytes incl. the ground pass's read of the kept points")
    tc = traffic_of("k_fa_points")
    roof_pc = roofline("k_project+k_fa_points", bpc_proj + bpc_curv, proj_ms + ktimes["k_fa_points"],
                       traffic=(tp + tc) if (tp is not None and tc is not None) else None,
                       note="north_star's projection+curvature figure: SURVEY.md 8(d) B_pc = 20 N + 24 HW + 29 S "
                            "over the two kernels' time")

    # the dominant kernel at SURVEY.md 8(d)'s own per-unit figure where it names one (feature
    # select B_fs = 25 S); the builder's wider model (incl. the VoxelGrid gathers) rides along
    if dom == "k_select_ring":
        split = ktimes.get("k_vox_pcl", 0.0) > 0.0
        ts, tv = traffic_of("k_select_ring"), traffic_of("k_vox_pcl")
        tsel = None if ts is None or (split and tv is None) else ts + (tv if split else 0.0)
        roof_dom = roofline(dom, 25 * csum["S"], ms=sel_ms, traffic=tsel,
                            note="SURVEY.md 8(d) B_fs = 25 S over the feature selection's time (k_select_ring "
                                 "+ k_vox_pcl, the PCL-order VoxelGrid); builder model incl. the less-flat "
                                 f"VoxelGrid gathers: {per[dom]:.4g} B per launch")
        roof_dom["traffic"] = tsel  # both kernels' PMC bytes, or null
        roof_dom["kernel"] = "k_select_ring+k_vox_pcl" if split else "k_select_ring"
        roof_dom["builder_model_frac"] = roofline(dom, ms=sel_ms)["frac"]
    else:
        roof_dom = roofline(dom)

    s2m = {}
    for mode_name in [m for m in args.s2m_modes.split(",") if m]:
        s2m[mode_name] = scan2map_leg(dev, mode_name, args.s2m_problems, args.s2m_steps, 1, dist,
                                      rank == 0 and not args.no_cpu and world == 1,
                                      min(args.cpu_seconds, 12.0), args.s2m_fixture)

    odo = {}
    for spec in [x for x in args.odo.split(",") if x]:
        lid, nb = spec.split(":")
        # frames: one continuous drive through warm-up, timed and profiled steps (no replay jump
        # from the last frame back to the first inside the measured region)
        odo[lid] = odometry_leg(dev, lid, int(nb), 2, 2 + args.s2m_steps, args.s2m_steps, 2, dist,
                                rank == 0 and not args.no_cpu and world == 1, min(args.cpu_seconds, 10.0))

    pc2 = pc2_decode_leg(dev, pts, off, args.s2m_steps * 4, dist) if args.pc2 else None

    lmap = None
    if args.map_keyframes > 0:
        lmap = local_map_leg(dev, args.map_keyframes, args.s2m_steps * 4, 2, dist,
                             rank == 0 and not args.no_cpu and world == 1, min(args.cpu_seconds, 8.0))

    mapping = None
    if args.mapping:
        mb, mw, ms_ = (int(x) for x in args.mapping.split(":"))
        mapping = mapping_leg(dev, mb, 4, mw, ms_, dist, rank == 0 and not args.no_cpu and world == 1,
                              min(args.cpu_seconds, 20.0))

    allred = None
    if args.allreduce_scans > 0:
        allred = scan2map_allreduce_leg(dev, args.allreduce_scans, args.s2m_steps, 1, dist or rccl1,
                                        rank == 0 and not args.no_cpu)

    if rank == 0:
        out = {
            "metric": "scans/sec (VLP-16 1800x16) at 1/2/4/8 GPUs; pose delta vs CPU ref",
            "value": round(value, 1),
            "unit": "scans/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "build_id": build_id(),
            "dtype": "fp32",
            "data": "synthetic (seeded ray-cast VLP-16 street scenes, 2% dropout, 1 cm noise)",
            "config": {"workload": "configs[1]: VLP-16 1800x16 projection + ground/cluster segmentation "
                                   "+ curvature/feature extraction, labels/indices bit-exact vs CPU",
                       "lidar": "VLP-16", "rings": H, "columns": W, "scans_per_gpu_per_step": B,
                       "distinct_clouds_per_gpu": args.distinct, "streams_per_gpu": nS,
                       "parallelism": f"scan-sharded x{world}"},
            "roofline": roof_dom,
            # north_star's kernel: the (fused) projection + range image + column ground pass
            "roofline_projection": roof_proj,
            "roofline_projection_curvature": roof_pc,
            "kernels_ms_per_step": {k: round(v, 4) for k, v in ktimes.items()},
            "pipeline_algorithmic_GBs": round(sum(per.values()) / (sum(ktimes.values()) * 1e-3) / 1e9, 1),
            "per_scan_mean": {k: round(v / B, 1) for k, v in csum.items() if k not in ("R", "M2")},
            "parity_spot_check_slot0": parity,
            "pose_delta": s2m.get("lm_applied", {}).get("pose_delta_max"),
            "scan2map": s2m,
            "scan2map_allreduce": allred,
            "odometry": odo,
            "local_map": lmap,
            "mapping": mapping,
            "pointcloud2_decode": pc2,
        }
        if not args.no_cpu and world == 1:
            scans = [pts[off[k]:off[k + 1]] for k in range(min(args.distinct, B))]
            out["cpu_baseline"] = cpu_baseline(scans, args.cpu_seconds)
            out["cpu_baseline"]["cpu"] = cpu_model()
            out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
            out["cpu_baseline_all_cores"] = cpu_baseline_all_cores(scans, min(args.cpu_seconds, 10.0))
            out["speedup_vs_cpu_all_cores"] = round(value / out["cpu_baseline_all_cores"]["value"], 1)
            out["cpu_pipeline_stages"] = cpu_stage_times(min(args.cpu_seconds, 10.0))
        print(json.dumps(out), flush=True)
    for p_ in pipes:
        p_.close()
    if dist:
        dist.destroy_process_group()
    elif rccl1 is not None:
        rccl1.destroy_process_group()


if __name__ == "__main__":
    main()
