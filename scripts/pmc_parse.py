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


def measured_build(sub):
    """The build id the profiled bench itself printed (its JSON line in <sub>.log): the library
    that was measured, not whatever the parsing process would load."""
    ids = set()
    for line in open(os.path.join(d, sub + ".log"), errors="replace"):
        line = line.strip()
        if line.startswith("{") and '"build_id"' in line:
            ids.add(json.loads(line)["build_id"])
    if len(ids) != 1:
        raise SystemExit(f"pmc_parse: {sub}.log names build ids {sorted(ids)}, expected exactly one")
    return ids.pop()


bid = {measured_build("fetch"), measured_build("write")}
if len(bid) != 1:
    raise SystemExit(f"pmc_parse: the FETCH_SIZE and WRITE_SIZE passes measured different builds {sorted(bid)}")
# the build these counters measured: bench.py reports the bytes only for the same build
print(json.dumps({"batch": batch, "build_id": bid.pop(), "kernels": out}, indent=1))
