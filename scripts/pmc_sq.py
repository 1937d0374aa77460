"""Per-kernel averages of the SQ counters of a rocprofv3 --pmc pass (scripts/pmc.sh SQ=1).

SQ_WAVE_CYCLES ~ WAIT_ANY (parked: s_waitcnt / barrier) + WAIT_INST_ANY (issue stall) +
ACTIVE_INST_ANY (issuing), all in quad-cycles (MI355X_MICROARCH.md, SQ counters). Prints the
per-dispatch means and those three as fractions of the wave cycles.

    python scripts/pmc_sq.py <dir of the sq pass>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("llsr::", "").split("<")[0]
        acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for k, cs in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    wc = m.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    m["frac_wait"] = round(m.get("SQ_WAIT_ANY", 0.0) / wc, 3)
    m["frac_issue_stall"] = round(m.get("SQ_WAIT_INST_ANY", 0.0) / wc, 3)
    m["frac_active"] = round(m.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 3)
    m["frac_valu"] = round(m.get("SQ_ACTIVE_INST_VALU", 0.0) / wc, 3)
    out[k] = m
print(json.dumps(out, indent=1))
