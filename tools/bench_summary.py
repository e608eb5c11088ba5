#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line: the headline, and per
perf_mode run the rate, kernel ms and quality (python tools/bench_summary.py LOG)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", d["metric"], d["value"], d["unit"], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"])
for k in ("roofline", "cpu_baseline"):
    if k in d and k == "cpu_baseline":
        print(k, {x: d[k][x] for x in ("value", "cores", "parity_bit_exact_on_sample") if x in d[k]})
pm = d.get("perf_mode", {})
for k, v in pm.items():
    if isinstance(v, dict) and "Mpatches_per_s" in v:
        cb = v.get("cpu_baseline", {})
        print(k, v["Mpatches_per_s"], v["kernel_ms_events"], "E", v["E_mean_evals_per_patch"], v["quality"],
              "valu" if "valu" in v["roofline"] else "", v["roofline"].get("valu", ""),
              "cpu_exact" if cb.get("parity_bit_exact_on_sample") else ("" if not cb else "CPU MISMATCH"))
    else:
        print(k, v)
for k in ("densify_e2e", "densify_e2e_fast", "densify_partitioned", "densify_partitioned_fast"):
    if k in d:
        print(k, d[k])
