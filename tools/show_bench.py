"""Print the headline and secondary numbers of a bench.py JSON line (GPU-run summaries)."""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("fusion step %.3f ms  %.4e updates/s  frac %.3f  (ms_per_step %.3f)  %s  F %s ms  valu-issue %s" % (
    r.get("step_ms", r.get("kernel_ms")), d["value"], r["frac"], d["ms_per_step"], r["kernel"], r.get("f_kernel_ms"),
    (r.get("companion") or {}).get("frac")))
print("digest %s expected %s match %s  rccl %s" % (d.get("logodds_digest"), d.get("digest_expected"),
                                                   d.get("digest_match"), d.get("rccl")))
s = d.get("secondary") or {}
if s:
    print("reverse %.3f ms/batch  forward %.3f ms/batch  costmap %.3f ms" % (
        s["reverse_ray_trace_fast"]["ms_per_batch"], s["forward_first_hits"]["ms_per_batch"],
        s["collision_cost_map"]["ms"]))
    for k, sub in (("reverse", s["reverse_ray_trace_fast"]), ("forward", s["forward_first_hits"]),
                   ("costmap", s["collision_cost_map"])):
        print("  %s digest_match %s" % (k, sub.get("digest_match")))
    rc = (s["reverse_ray_trace_fast"].get("cpu_baseline") or {})
    print("  reverse cpu pose0_list_match %s" % rc.get("pose0_list_match"))
for k in ("cpu_baseline", "cpu_baseline_multicore", "cpu_baseline_reference"):
    c = d.get(k)
    if c:
        print("%s: %.4e %s cores %s  %s" % (k, c["value"], c["unit"], c["cores"], c["sample"][:120]))
