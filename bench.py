"""bench.py — scans/sec of the MI355X LeGO-LOAM-SR hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1]): synthetic VLP-16 1800x16 scans through projection + ground /
cluster segmentation (ImageProjection) + curvature / feature extraction (FeatureAssociation
feature stage), labels / feature indices bit-exact vs the CPU path. A "step" is one pass of the
hot path over one batch of B scans per GPU that is already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

N > 1 is launched by torch.distributed.run (one rank per GPU). Scans are batch-sharded: every
rank processes its own B scans with no data-path collective (weak scaling); ranks only meet at the
barriers around the timed region and for the max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lego-loam-sr_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


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
        "k_fa_points": 62 * S,
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
    ora = oracle_py.Oracle(_abi.config_for("vlp16"))
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="scans per GPU per step")
    ap.add_argument("--distinct", type=int, default=16, help="distinct synthetic scans per rank")
    ap.add_argument("--streams", type=int, default=2,
                    help="handles/HIP streams used round-robin, so consecutive batches overlap")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
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

    from llsr import Pipeline, default_config, synth
    cfg = default_config("vlp16")
    H, W = cfg.num_vertical_scans, cfg.num_horizontal_scans
    B = args.batch
    pts, off = synth.make_batch(B, "vlp16", distinct=args.distinct, seed0=1 + 1000 * rank)
    d_pts = torch.from_numpy(pts).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    nS = max(1, args.streams)
    pipes = [Pipeline(cfg, device=dev, max_batch=B, max_points=int(np.diff(off).max())) for _ in range(nS)]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nS - 1)]
    pipe = pipes[0]
    torch.cuda.synchronize(dev)

    def step(k):
        pipes[k % nS].process_batch(d_pts.data_ptr(), d_off.data_ptr(), B, streams[k % nS].cuda_stream)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    pipe.set_profiling(True)
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
    ktimes = pipe.kernel_times()  # ms per batch, HIP events on the launch stream
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
    if ktimes.get("k_gather_column", 1.0) == 0.0:  # fused projection kernel (H*W fits LDS)
        per["k_project"] += per["k_gather_column"]
        per["k_gather_column"] = 0.0
    dom = max((k for k in ktimes if k != "init"), key=lambda k: ktimes[k])
    achieved = per[dom] / (ktimes[dom] * 1e-3) / 1e9
    total_scans = B * args.steps * world
    value = total_scans / el
    parity = None
    if rank == 0 and not args.no_cpu:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_py
        from _compare import compare
        # slot 0 of handle 0 has seen every nS-th batch of the same cloud: replay that history
        ora = oracle_py.Oracle(cfg)
        n0 = len(range(0, args.warmup, nS)) + len(range(0, args.steps, nS))
        for _ in range(n0):
            o = ora.process(pts[off[0]:off[1]])
        parity = not compare(r0, o)

    # PMC-measured HBM bytes per launch (scripts/pmc.sh, committed under profiles/), per scan
    # scaled to this batch size; null when no measurement for this kernel exists.
    traffic = None
    tfile = os.environ.get("LLSR_TRAFFIC_JSON", os.path.join(REPO, "profiles", "traffic_latest.json"))
    if os.path.exists(tfile):
        t = json.load(open(tfile))
        rec = t.get("kernels", {}).get(dom)
        if rec and t.get("batch"):
            traffic = rec["hbm_bytes"] / t["batch"] * B

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
            "dtype": "fp32",
            "data": "synthetic (seeded ray-cast VLP-16 street scenes, 2% dropout, 1 cm noise)",
            "config": {"workload": "configs[1]: VLP-16 1800x16 projection + ground/cluster segmentation "
                                   "+ curvature/feature extraction, labels/indices bit-exact vs CPU",
                       "lidar": "VLP-16", "rings": H, "columns": W, "scans_per_gpu_per_step": B,
                       "distinct_clouds_per_gpu": args.distinct, "streams_per_gpu": nS,
                       "parallelism": f"scan-sharded x{world}"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "algorithmic_bytes_per_launch": per[dom], "avg_launch_ms": round(ktimes[dom], 4)},
            "kernels_ms_per_step": {k: round(v, 4) for k, v in ktimes.items()},
            "pipeline_algorithmic_GBs": round(sum(per.values()) / (sum(ktimes.values()) * 1e-3) / 1e9, 1),
            "per_scan_mean": {k: round(v / B, 1) for k, v in csum.items() if k not in ("R", "M2")},
            "parity_spot_check_slot0": parity,
            "pose_delta": None,
        }
        if not args.no_cpu and world == 1:
            scans = [pts[off[k]:off[k + 1]] for k in range(min(args.distinct, B))]
            out["cpu_baseline"] = cpu_baseline(scans, args.cpu_seconds)
            out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    for p_ in pipes:
        p_.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
