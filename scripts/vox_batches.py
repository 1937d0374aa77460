"""A short GPU workload for kernel-level profiling of the feature stage: N batches of B VLP-16 scans
(16 distinct clouds cycled, as the bench's headline) through Pipeline.process_batch on one stream.

    python scripts/vox_batches.py [N] [B]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-sr_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from llsr import Pipeline, default_config, synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 6
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
cfg = default_config("vlp16")
pts, off = synth.make_batch(B, "vlp16", distinct=16)
d_pts, d_off = torch.from_numpy(pts).cuda(), torch.from_numpy(off).cuda()
pipe = Pipeline(cfg, max_batch=B, max_points=int(np.diff(off).max()))
for _ in range(N):
    pipe.process_batch(d_pts.data_ptr(), d_off.data_ptr(), B)
torch.cuda.synchronize()
print("ok", N, B)
