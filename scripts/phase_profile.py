"""Attribute kernel time to phases: run one batch, then re-launch selected kernels with an
early exit at each phase boundary (diagnostic launches; their outputs are meaningless)."""
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
pts, off = synth.make_batch(B, lidar, distinct=int(os.environ.get("DISTINCT", "16")))
d_pts, d_off = torch.from_numpy(pts).cuda(), torch.from_numpy(off).cuda()
pipe = Pipeline(cfg, max_batch=B, max_points=int(np.diff(off).max()))
pipe.set_voxel_order(int(os.environ.get("VOXEL_ORDER", "1")))  # 1 = LLSR_VOXEL_ORDER_PCL
for _ in range(3):
    pipe.process_batch(d_pts.data_ptr(), d_off.data_ptr(), B)
pipe.set_profiling(True)
for _ in range(3):  # kernel_times() averages over the profiled batches (bench.py's prof pass)
    pipe.process_batch(d_pts.data_ptr(), d_off.data_ptr(), B)
res = {"kernels": pipe.kernel_times()}
names = {3: "k_ground_add", 4: "k_ground_elev_ransac", 5: "k_label", 6: "k_segment", 7: "k_fa_points",
         8: "k_select_ring", 9: "k_vox_pcl", 10: "k_fa_concat", 11: "k_dbscan_adj", 12: "k_dbscan_merge"}
names[1] = "k_project_fused"
todo = []
for x in os.environ.get("PHASES", "8:8").split(","):  # "k:n" = phases 0..n-1, "k:a:b" = a..b-1
    f = [int(v) for v in x.split(":")]
    todo.append((f[0], range(f[1]) if len(f) == 2 else range(f[1], f[2])))
for k, phases in todo:
    res[names[k]] = {p: round(pipe.debug_phase_ms(k, p, 5), 4) for p in phases}
print(json.dumps(res))
