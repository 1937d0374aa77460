"""Phase attribution of k_s2s_lm from the diagnostic build (make -C lego-loam-sr_amd prof): runs
the bench's odometry batches (two continuous drives, 2 warm-up + 4 measured frames) with LLSR_LIB=libllsr_prof.so
and reports, over the slots and the four frames, the mean per-problem
wall time of the kNN-1 search (shells / LDS scan, with the block scans for queries the shells
left open) for surf / corner, the Jacobian rows, B (ordered sums), C (solve) and the tripod walks
for corner / surf, in us.

    python scripts/s2s_prof.py [vlp16|hdl64e] [B]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LLSR_LIB"] = os.path.join(REPO, "lego-loam-sr_amd", os.environ.get("S2S_PROF_LIB", "libllsr_prof.so"))
sys.path.insert(0, os.path.join(REPO, "lego-loam-sr_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from llsr import Pipeline, _abi, default_config, synth  # noqa: E402

lidar = sys.argv[1] if len(sys.argv) > 1 else "vlp16"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
cfg = default_config(lidar, 2048 if lidar == "hdl64e" else None)
cfg.mode = _abi.LLSR_MODE_LM_APPLIED
# the bench's odometry leg: 2 continuous drives
NF = 6  # 2 warm-up frames, then 4 measured, one continuous drive (no jump back)
seqs = [[synth.make_scan(1 + 64 * q + k, lidar, motion=True) for k in range(NF)] for q in range(2)]
pipe = Pipeline(cfg, max_batch=B, max_points=cfg.num_vertical_scans * cfg.num_horizontal_scans)
batches = []
for k in range(NF):
    scans = [seqs[b % 2][k] for b in range(B)]
    off = np.zeros(B + 1, np.int64)
    off[1:] = np.cumsum([len(a) for a in scans])
    batches.append((torch.from_numpy(np.concatenate(scans)).cuda(), torch.from_numpy(off).cuda()))
rows = []
per = {}  # (frame, sequence) -> rows
for n in range(6):  # 2 warm-up batches, then one of each frame
    d_pts, d_off = batches[n]
    torch.cuda.synchronize()
    pipe.odometry_batch(d_pts.data_ptr(), d_off.data_ptr(), B)
    torch.cuda.synchronize()
    if n < 2:
        continue
    prof = np.zeros((B, 8), np.float32)
    pipe.debug_s2s_prof(prof)
    for b in list(range(0, B, max(1, B // 64))) + [1, 3]:
        f = pipe.odometry_fetch(b)
        t = prof[b] / 100.0  # 100 MHz ticks -> us (problem b of the launch = slot b)
        rows.append(list(t[:7]) + [f["lm"]["surf_iterations"], f["lm"]["corner_iterations"],
                                   f["lm"]["n_surf_corr"], f["lm"]["n_corner_corr"], float(prof[b, 7])])
        per.setdefault((n, b % 2), []).append(rows[-1])
r = np.array(rows)
print(json.dumps({"lidar": lidar, "B": B,
                  "us_per_problem": dict(zip(["knn_surf", "knn_corner", "A_rows", "B_sums", "C_solve",
                                              "walks_corner", "walks_surf"], r[:, :7].mean(0).round(1).tolist())),
                  "iterations": dict(zip(["surf", "corner"], r[:, 7:9].mean(0).round(1).tolist())),
                  "slowest_problem": {"us": dict(zip(["knn_surf", "knn_corner", "A_rows", "B_sums", "C_solve",
                                                      "walks_corner", "walks_surf"],
                                                     r[r[:, :7].sum(1).argmax(), :7].round(1).tolist())),
                                      "iterations": r[r[:, :7].sum(1).argmax(), 7:9].tolist()},
                  "correspondences": dict(zip(["surf", "corner"], r[:, 9:11].mean(0).round(1).tolist())),
                  "per_frame_sequence": {f"frame {k[0]} seq {k[1]}": {
                      "us": dict(zip(["knn_surf", "knn_corner", "A_rows", "B_sums", "C_solve", "walks_corner", "walks_surf"],
                                     np.array(v)[:, :7].mean(0).round(1).tolist())),
                      "iterations": np.array(v)[:, 7:9].mean(0).round(1).tolist(),
                      "shell_fallback_queries": float(np.array(v)[:, 11].mean())} for k, v in sorted(per.items())}}))
