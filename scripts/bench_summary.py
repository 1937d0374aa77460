"""Summarise a bench.py output file (the JSON line is the last line; RCCL may print a banner first)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"value {d['value']} scans/s, {d['ms_per_step']} ms/step, build {d.get('build_id')}")
print(f"roofline {r['kernel']} frac {r['frac']} (builder {r.get('builder_model_frac')}) traffic {r['traffic']}; "
      f"projection {d['roofline_projection']['frac']}, projection+curvature {d['roofline_projection_curvature']['frac']}")
print("kernels", sorted(d["kernels_ms_per_step"].items(), key=lambda x: -x[1]))
for k, v in d["odometry"].items():
    print(f"odometry {k}: {v['value']} scans/s, lm {v['kernels_ms_per_step'].get('k_s2s_lm')} ms, surf it mean "
          f"{v.get('surf_iterations_mean')} max {v.get('surf_iterations_max')}, it {v['lm_iterations_mean']}, cpu "
          f"{v.get('cpu_baseline', {}).get('value')}, pose delta {v.get('pose_delta_max')}")
m = d.get("mapping") or {}
print(f"mapping {m.get('value')} bit-exact {m.get('bit_exact_slot0')} cpu {m.get('cpu_baseline', {}).get('value')} "
      f"all-core {m.get('cpu_baseline_all_cores', {}).get('value')}")
for k, v in d["scan2map"].items():
    print(f"scan2map {k}: {v['value']} problems/s, grid {v['grid_build_ms_per_step']} iterate {v['iterate_ms_per_step']} "
          f"ms, pose delta {v.get('pose_delta_max')}, cpu {v.get('cpu_baseline', {}).get('value')}")
a = d.get("scan2map_allreduce") or {}
print(f"allreduce {a.get('value')}, local_map {d['local_map']['value'] if d.get('local_map') else None}, "
      f"pc2 {d['pointcloud2_decode']['value'] if d.get('pointcloud2_decode') else None}")
if "cpu_baseline" in d:
    print(f"cpu {d['cpu_baseline']['value']} ({d['cpu_baseline']['cores']} core), all-core "
          f"{d['cpu_baseline_all_cores']['value']} ({d['cpu_baseline_all_cores']['cores']}), full host "
          f"{d['cpu_baseline_all_cores'].get('full_host_extrapolated')} of {d['cpu_baseline_all_cores'].get('host_cpus')}")
