"""How far the FA less-flat VoxelGrid's summation order moves the odometry: one drive through the
oracle's odometry restatement twice, in PCL's std::sort order and in input order, and the largest
transformSum difference per frame (CPU only; the oracle is the checker, this is its analysis).

    python scripts/voxel_order_drift.py [lidar] [frames] [first_seed] > profiles/<name>.json
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-sr_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle_py  # noqa: E402
from llsr import _abi, default_config, synth  # noqa: E402

lidar = sys.argv[1] if len(sys.argv) > 1 else "hdl64e"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 12
seed0 = int(sys.argv[3]) if len(sys.argv) > 3 else 1
cfg = default_config(lidar, 2048 if lidar == "hdl64e" else None)
cfg.mode = _abi.LLSR_MODE_LM_APPLIED
pcl = oracle_py.OracleOdometry(cfg, pcl_voxel_order=True)
inp = oracle_py.OracleOdometry(cfg, pcl_voxel_order=False)
rows = []
for k in range(frames):
    pts = synth.make_scan(seed0 + k, lidar, motion=True)
    a, b = pcl.process(pts), inp.process(pts)
    d = float(np.abs(np.asarray(a["transform_sum"], np.float64) - np.asarray(b["transform_sum"], np.float64)).max())
    rows.append({"frame": k, "transform_sum_delta_max": d})
print(json.dumps({"lidar": lidar, "frames": frames, "first_seed": seed0, "drive": "synth.make_scan(seed, motion=True)",
                  "max_transform_sum_delta": max(r["transform_sum_delta_max"] for r in rows), "per_frame": rows},
                 indent=1))
