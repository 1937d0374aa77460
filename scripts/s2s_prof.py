"""Phase attribution of k_s2s_lm from the diagnostic build (make -C lego-loam-sr_amd prof): runs
the odometry batch with LLSR_LIB=libllsr_prof.so and reports, over the slots, the mean per-problem
wall time of the kNN search (shells / LDS scan + ring search) for surf / corner, the block
scans for queries the shells left open, the Jacobian rows, B (ordered sums) and C (solve), in us.

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
seqs = [[synth.make_scan(1 + 64 * q + k, lidar) for k in range(3)] for q in range(2)]
pipe = Pipeline(cfg, max_batch=B, max_points=cfg.num_vertical_scans * cfg.num_horizontal_scans)
for k in range(3):
    scans = [seqs[b % 2][k] for b in range(B)]
    off = np.zeros(B + 1, np.int64)
    off[1:] = np.cumsum([len(a) for a in scans])
    d_pts, d_off = torch.from_numpy(np.concatenate(scans)).cuda(), torch.from_numpy(off).cuda()
    torch.cuda.synchronize()
    pipe.odometry_batch(d_pts.data_ptr(), d_off.data_ptr(), B)
    torch.cuda.synchronize()
rows = []
for b in range(0, B, max(1, B // 64)):
    f = pipe.odometry_fetch(b)
    t = f["lm"]["transform_cur"] / 100.0  # 100 MHz ticks -> us
    rows.append(list(t[:6]) + [f["lm"]["surf_iterations"], f["lm"]["corner_iterations"]])
r = np.array(rows)
print(json.dumps({"lidar": lidar, "B": B,
                  "us_per_problem": dict(zip(["knn_surf", "knn_corner", "A_rows", "B_sums", "C_solve",
                                              "knn_fallback"], r[:, :6].mean(0).round(1).tolist())),
                  "iterations": dict(zip(["surf", "corner"], r[:, 6:].mean(0).round(1).tolist()))}))
