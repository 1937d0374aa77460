"""Per-kernel HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE rocprofv3 passes.

MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half
the bytes of a wide coalesced streaming read, so it is doubled here (an upper bound for kernels
whose reads are not 16 B/lane streams; uncalibrated for other widths). Output: {"batch": B,
"kernels": {name: {fetch_bytes_x2, write_bytes, hbm_bytes, launches}}} — bench.py scales
hbm_bytes by its own batch size into roofline.traffic.

    python scripts/pmc_parse.py <dir with fetch/ and write/ passes> <batch>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1024


def load(sub, counter):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("llsr::", "")
            name = name.split("<")[0]
            acc[name].append(float(row["Counter_Value"]))
    return acc


fetch, write = load("fetch", "FETCH_SIZE"), load("write", "WRITE_SIZE")
out = {}
for k in sorted(set(fetch) | set(write)):
    fv, wv = fetch.get(k, []), write.get(k, [])
    f = (sum(fv) / len(fv) if fv else 0.0) * 1024 * 2
    w = (sum(wv) / len(wv) if wv else 0.0) * 1024
    out[k] = {"fetch_bytes_x2": f, "write_bytes": w, "hbm_bytes": f + w, "launches": max(len(fv), len(wv))}
# the build these counters measured: bench.py reports the bytes only for the same build
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lego-loam-sr_amd"))
import llsr  # noqa: E402
print(json.dumps({"batch": batch, "build_id": llsr.build_id(), "kernels": out}, indent=1))
