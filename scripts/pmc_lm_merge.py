"""Merge scripts/pmc_lm.sh's two legs into the profiles/traffic_lm_latest.json format: per LM
kernel and leg the HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, scripts/pmc_parse.py) and
the SQ split (scripts/pmc_sq.py).

    python scripts/pmc_lm_merge.py <pmc_lm output dir> <source tag>
"""
import json
import os
import sys

d, src = sys.argv[1], sys.argv[2]


def load(leg):
    t = json.load(open(os.path.join(d, leg, "traffic.json")))["kernels"]
    sq = json.load(open(os.path.join(d, leg, "sq.json")))
    return t, sq


want = {"A": [("k_s2m_iter", None, "scan2map lm_applied", 256), ("k_s2m_solve", None, "scan2map lm_applied", 256),
              ("k_s2s_lm", "odometry vlp16", "odometry vlp16", 1024)],
        "B": [("k_s2s_lm", "odometry hdl64e", "odometry hdl64e", 512)]}
out = {"source": f"scripts/pmc_lm.sh ({src}): rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / 8 SQ counters, one "
                 "pass each, kernel-trace only; leg A = scan2map lm_applied (P 256) + VLP-16 odometry (1024 "
                 "scans), leg B = HDL-64E odometry (512 scans)",
       "note": "FETCH_SIZE doubled per the gfx950 note (scripts/pmc_parse.py); bytes per launch averaged over "
               "the pass's launches", "kernels": {}}
ids = {json.load(open(os.path.join(d, leg, "traffic.json"))).get("build_id") for leg in want}
assert len(ids) == 1, ids
out["build_id"] = ids.pop()
for leg, items in want.items():
    t, sq = load(leg)
    for k, key_leg, leg_name, problems in items:
        if k not in t:
            continue
        rec = {"leg": leg_name, "problems": problems, "hbm_bytes_per_launch": t[k]["hbm_bytes"],
               "fetch_bytes_x2": t[k]["fetch_bytes_x2"], "write_bytes": t[k]["write_bytes"],
               "launches": t[k]["launches"]}
        if k in sq:
            rec["sq"] = {x: sq[k][x] for x in ("frac_wait", "frac_issue_stall", "frac_active", "frac_valu") if x in sq[k]}
        if key_leg:
            rec["leg_key"] = key_leg
        out["kernels"][f"{k}@{key_leg}" if key_leg else k] = rec
print(json.dumps(out, indent=1))
