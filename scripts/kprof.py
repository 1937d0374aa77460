"""Single-stream per-kernel device times of the IP + feature pipeline (HIP events between the
kernels of each batch, llsr_kernel_times_ms) and phase attribution of selected kernels by
early-exit re-launches (llsr_debug_phase_ms; diagnostic launches, outputs meaningless).

    python scripts/kprof.py [vlp16|hdl64e] [B]
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-sr_amd"))
from llsr import Pipeline, default_config, synth  # noqa: E402

lidar = sys.argv[1] if len(sys.argv) > 1 else "vlp16"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
cfg = default_config(lidar, 2048 if lidar == "hdl64e" else None)
pts, off = synth.make_batch(B, lidar, distinct=8)
d_pts, d_off = torch.from_numpy(pts).cuda(), torch.from_numpy(off).cuda()
pipe = Pipeline(cfg, max_batch=B, max_points=int(np.diff(off).max()))
for _ in range(3):
    pipe.process_batch(d_pts.data_ptr(), d_off.data_ptr(), B)
pipe.set_profiling(True)
for _ in range(5):
    pipe.process_batch(d_pts.data_ptr(), d_off.data_ptr(), B)
res = {"lidar": lidar, "B": B, "kernels_ms": {k: round(v, 4) for k, v in pipe.kernel_times().items()}}
cnt = pipe.batch_counts(B)
res["per_scan_mean"] = dict(zip(["N", "S", "O", "M", "sharp", "F", "L", "K"], cnt.mean(axis=0).round(1).tolist()))
res["M_max"] = int(cnt[:, 3].max())
phases = {1: ("k_project_fused", range(0, 3)), 8: ("k_select_ring", range(0, 8))}
for k, (name, ph) in phases.items():
    res[name + "_phase_ms"] = {p: round(pipe.debug_phase_ms(k, p, 5), 4) for p in ph}
print(json.dumps(res))
