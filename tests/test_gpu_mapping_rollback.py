"""GPU: llsr_mapping_batch's error contract (include/llsr.h: an error from the MapOptimization part of
a call, after the odometry advanced, leaves every slot's MapOptimization members as before the
call — the snapshot / restore in llsr_capi.hip's llsr_mapping_batch).

No input makes MapOptimization fail on purpose, so the diagnostics build (libllsr_prof.so, built
with LLSR_S2S_PROF by `make`) fails it once on request: LLSR_MO_FAIL_AT=k fails the call in which
slot 0 reaches MapOptimization frame k, after that call's keyframes were added, so the restore has
keyframes, key poses, every pose, the LM report and the local-map selection to undo. The drive runs
in a child process (the library is chosen at import) and reports what it fetched.

Bar: the failing call raises; every slot's fetched MapOptimization fields (mo_frames, keyframes,
lm_ran, query sizes, the four poses, the LM and map reports) and its key poses equal those before
the call; the next call succeeds and advances mo_frames by one."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "lego-loam-sr_amd", "libllsr_prof.so")

CHILD = r"""
import json, sys
import numpy as np, torch
sys.path.insert(0, sys.argv[1])
from llsr import LlsrError, Pipeline, _abi, default_config, synth
cfg = default_config("vlp16")
cfg.mode = _abi.LLSR_MODE_LM_APPLIED
seeds = [3, 40]
pipe = Pipeline(cfg, max_batch=len(seeds), max_points=cfg.num_vertical_scans * cfg.num_horizontal_scans)
pipe.mapping_init(_abi.LLSR_MODE_LM_APPLIED)
def state(b):
    f = pipe.mapping_fetch(b)
    f.pop("frames")  # the odometry's frame count: advanced by the failing call, not a MapOptimization member
    out = {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in f.items()}
    out["keyposes"] = pipe.mapping_keyposes(b).tolist()
    return out
res = {"failed_at": None, "before": None, "after": None, "next_mo_frames": None, "mo_before": None}
for k in range(8):
    scans = [synth.make_scan(s0 + k, "vlp16", motion=True) for s0 in seeds]
    off = np.zeros(len(scans) + 1, np.int64)
    off[1:] = np.cumsum([len(s) for s in scans])
    d_pts, d_off = torch.from_numpy(np.concatenate(scans)).cuda(), torch.from_numpy(off).cuda()
    torch.cuda.synchronize()
    snap = [state(b) for b in range(len(seeds))]
    try:
        pipe.mapping_batch(d_pts.data_ptr(), d_off.data_ptr(), len(scans))
    except LlsrError as e:
        res["failed_at"] = k
        res["error"] = str(e)
        res["before"] = snap
        res["after"] = [state(b) for b in range(len(seeds))]
        continue
    if res["failed_at"] is not None and res["next_mo_frames"] is None:
        res["mo_before"] = [s["mo_frames"] for s in res["after"]]
        res["next_mo_frames"] = [pipe.mapping_fetch(b)["mo_frames"] for b in range(len(seeds))]
print(json.dumps(res, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o)))
"""


def test_mapping_batch_restores_mapoptimization_on_error(require_gpu):
    assert os.path.exists(PROF), "libllsr_prof.so missing: run make -C lego-loam-sr_amd"
    env = dict(os.environ, LLSR_LIB=PROF, LLSR_MO_FAIL_AT="3")
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(REPO, "lego-loam-sr_amd")], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["failed_at"] is not None, "the injected failure never fired"
    assert "injected MapOptimization failure" in res["error"]
    for b, (pre, post) in enumerate(zip(res["before"], res["after"])):
        assert pre["keyframes"] >= 1, f"slot {b}: nothing to roll back"
        for key in pre:  # compared as JSON text: NaN fields compare equal to themselves
            assert json.dumps(post[key]) == json.dumps(pre[key]), f"slot {b}: {key} changed by the failed call"
    assert res["next_mo_frames"] == [m + 1 for m in res["mo_before"]]
