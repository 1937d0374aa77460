"""Print the key numbers of a gpu_check.sh run directory (gpurun_out/<tag>)."""
import json
import os
import sys

d = sys.argv[1]
print(open(os.path.join(d, "steps.log")).read().strip().replace("\n", " | "))
t = os.path.join(d, "pytest_gpu.log")
if os.path.exists(t):
    lines = open(t).read().strip().splitlines()
    print("pytest:", lines[-1] if lines else "")
    for ln in lines:
        if ln.startswith("FAILED") or ln.startswith("E  "):
            print("  ", ln[:300])
b = os.path.join(d, "bench.log")
if os.path.exists(b):
    for ln in open(b):
        if ln.startswith("{"):
            j = json.loads(ln)
            print("value", j["value"], j["unit"], "ms/step", j["ms_per_step"], "parity", j["parity_spot_check_slot0"],
                  "speedup", j.get("speedup_vs_cpu"), "cpu", round(j.get("cpu_baseline", {}).get("value", 0), 1))
            print("roofline", j["roofline"])
            print("kernels", j["kernels_ms_per_step"])
            print("pipeline GB/s", j["pipeline_algorithmic_GBs"])
s = os.path.join(d, "prof", "run_kernel_stats.csv")
if os.path.exists(s):
    for ln in open(s).read().splitlines()[:14]:
        f = ln.split('","')
        print("  ", f[0][:60].strip('"'), f[1] if len(f) > 1 else "", f[3] if len(f) > 3 else "")
