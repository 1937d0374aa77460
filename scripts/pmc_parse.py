"""Per-kernel HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE rocprofv3 passes.

MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half
the bytes of a wide coalesced streaming read, so it is doubled here (an upper bound for kernels
whose reads are not 16 B/lane streams; uncalibrated for other widths)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]


def load(sub, counter):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("llsr::", "")
            name = name.split("<")[0]
            acc[name].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch, write = load("fetch", "FETCH_SIZE"), load("write", "WRITE_SIZE")
out = {}
for k in sorted(set(fetch) | set(write)):
    f, w = fetch.get(k, 0.0) * 1024 * 2, write.get(k, 0.0) * 1024
    out[k] = {"fetch_bytes_x2": f, "write_bytes": w, "hbm_bytes": f + w}
print(json.dumps(out, indent=1))
