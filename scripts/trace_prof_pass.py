"""Per-kernel durations of bench.py's single-stream profiling pass, read from a rocprofv3
kernel trace of the same bench command: for each IP / feature kernel, the dispatches number
[warmup + steps, warmup + steps + prof_batches) in start order (the main leg runs first), next to
the average over all of that kernel's dispatches (which includes launches sharing the GPU with
other streams). These are the durations bench.py's roofline divides by (its HIP events).

    python scripts/trace_prof_pass.py <run_kernel_trace.csv> <warmup> <steps> <prof_batches>
"""
import csv
import json
import sys
from collections import defaultdict

path, W, K, P = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
KERNELS = ("k_project_fused", "k_ground_add", "k_ground_elev_ransac", "k_label", "k_segment", "k_fa_points",
           "k_select_ring", "k_vox_pcl", "k_fa_concat", "k_dbscan_adj", "k_dbscan_merge")
runs = defaultdict(list)
for row in csv.DictReader(open(path)):
    name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("llsr::", "").split("<")[0]
    if name in KERNELS:
        runs[name].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
out = {}
for name in KERNELS:
    d = sorted(runs.get(name, []))
    sel = d[W + K:W + K + P]
    out[name] = {"dispatches": len(d),
                 "avg_ms_all": round(sum(e - s for s, e in d) / max(1, len(d)) / 1e6, 4),
                 "avg_ms_profiling_pass": round(sum(e - s for s, e in sel) / max(1, len(sel)) / 1e6, 4)}
print(json.dumps(out, indent=1))
