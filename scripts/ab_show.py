"""Print the odometry / headline legs of an A/B run (scripts/ab_odo.sh): python scripts/ab_show.py DIR"""
import json
import os
import sys

d = sys.argv[1]
for name in ("base", "new", "new2"):
    f = os.path.join(d, name + ".json")
    if not os.path.exists(f):
        continue
    j = json.loads(open(f).read().strip().splitlines()[-1])
    line = [f"{name:5s} headline {j['value']:.0f}"]
    for lid, v in j.get("odometry", {}).items():
        k = v["kernels_ms_per_step"]
        line.append(f"{lid} {v['value']:.0f} scans/s lm {k.get('k_s2s_lm')} ms surf_it {v.get('surf_iterations_mean')} "
                    f"it {v['lm_iterations_mean']:.1f}")
    for mode, v in (j.get("scan2map") or {}).items():
        line.append(f"s2m {mode} {v['value']:.0f} grid {v['grid_build_ms_per_step']} it {v['iterate_ms_per_step']}")
    if j.get("mapping"):
        line.append(f"mapping {j['mapping']['value']:.0f}")
    print(" | ".join(line))
