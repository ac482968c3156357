"""Print the headline and secondary numbers of a bench.py JSON line (GPU-run summaries)."""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("fusion %.3f ms/launch  %.4e updates/s  frac %.3f  step %.3f ms  %s" % (r["kernel_ms"], d["value"], r["frac"],
                                                                           d["ms_per_step"], r["kernel"]))
s = d.get("secondary") or {}
if s:
    print("reverse %.3f ms/batch  forward %.3f ms/batch  costmap %.3f ms" % (
        s["reverse_ray_trace_fast"]["ms_per_batch"], s["forward_first_hits"]["ms_per_batch"],
        s["collision_cost_map"]["ms"]))
