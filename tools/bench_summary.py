"""One-screen summary of a bench.py JSON line (the headline, roofline, CPU baselines and the secondary legs).
usage: python tools/bench_summary.py LOG"""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    r = d.get("roofline", {})
    print({k: d.get(k) for k in ("value", "ms_per_step", "p50_batch_latency_ms", "n_gpus")})
    print("roofline frac", r.get("frac"), "executed", r.get("executed_frac"), "valu_busy", r.get("valu_busy"),
          "kernel", r.get("executed", {}).get("kernel"), r.get("executed", {}).get("unmeasured"))
    print("solver", d.get("solver"))
    for k in ("cpu_baseline", "cpu_backend", "cpu_reference"):
        c = d.get(k, {})
        print(k, c.get("value"), "cores", c.get("cores"), "share", (c.get("share") or {}).get("value"),
              (c.get("share") or {}).get("cores"))
    for k in ("nlp_sqp", "inflight"):
        print(k, {a: b for a, b in d.get(k, {}).items() if not isinstance(b, (dict, list, str))})
    cl = d.get("closed_loop", {})
    print("closed_loop", {k: cl.get(k) for k in ("egos", "ranks", "ego_steps_per_s", "seconds")},
          cl.get("checks_passed", {}).get("passed"))
    p = d.get("plan", {})
    print("plan", {k: p.get(k) for k in ("value", "ms_per_step")}, "cpu", p.get("cpu_baseline", {}).get("value"),
          p.get("cpu_baseline", {}).get("cores"), "parity", p.get("parity_sample"))
    f = p.get("fleet", {})
    print("fleet", {k: f.get(k) for k in ("seconds", "plans_per_s", "chunks", "checks_passed")})
