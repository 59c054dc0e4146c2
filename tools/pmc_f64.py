"""Summarise the executed-work PMC pass (tools/gpu/pmc_f64.sh) per solver kernel.

Per launch of each kernel (mode XO / IPM / FULL / ONE, template <OBS, G, MODE, NT>):
- FP64 VALU instructions by class (SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64, summed over all waves);
- an upper bound on executed FP64 flops: (2 FMA + MUL + ADD + TRANS) x 64 lanes.  The bound counts every
  lane of every issued instruction; the recursions run under an exec mask of 5 or 10 lanes, so the real
  count is lower;
- VALU-busy: SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (both in quad-cycles, MI355X_MICROARCH.md), the fraction
  of resident-wave time spent issuing VALU instructions.
The kernel-stats CSV of the same command (rocprofv3 --kernel-trace --stats, its own run) is required: the
flops are divided by each kernel's average duration to give executed TFLOP/s and its fraction of the 78.6 TF
FP64 peak, and every counted kernel must find its duration there (the script stops otherwise, so a summary
without durations cannot be written).

  python tools/pmc_f64.py C2 STATS.csv     ->  gpurun_out/pmc_f64_C2.csv and one JSON line per kernel
  python tools/pmc_f64.py plan STATS.csv   ->  the planner kernel (tools/gpu/plan_pmc_f64.sh)
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 78.6
MODES = {"0": "FULL", "1": "XO", "2": "IPM", "3": "ONE"}
CTRS = ["SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64",
        "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"]


def kernel_key(name):
    if "plan_chunk_kernel" in name:
        return "plan_chunk_kernel"
    if "mpc_solve_kernel" not in name:
        return None
    try:
        targs = [a.strip() for a in name.split("<", 1)[1].split(">")[0].split(",")]
        return f"mpc_solve_kernel<{','.join(targs)}> {MODES.get(targs[2], targs[2])}"
    except Exception:
        return name[:60]


def load_counters(d):
    per = {}       # key -> {dispatch -> {counter: value}}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = kernel_key(row.get("Kernel_Name", ""))
            if k is None:
                continue
            disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
            c = per.setdefault(k, {}).setdefault(disp, {})
            c[row["Counter_Name"]] = c.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return per


def load_stats(path):
    out = {}
    if not path or not os.path.exists(path):
        return out
    for row in csv.DictReader(open(path)):
        k = kernel_key(row.get("Name", ""))
        if k is not None:
            out[k] = (float(row["AverageNs"]) * 1e-9, float(row["TotalDurationNs"]) * 1e-9)
    return out


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
    if len(sys.argv) < 3:
        raise SystemExit("usage: pmc_f64.py CONFIG STATS.csv (the kernel-stats CSV of the same command)")
    stats = load_stats(sys.argv[2])
    if not stats:
        raise SystemExit(f"no solver kernel in {sys.argv[2]}")
    per = load_counters(os.path.join(ROOT, "gpurun_out", f"pmc_f64_{cfg}"))
    if not per:
        raise SystemExit("no counter rows found")
    missing = sorted(set(per) - set(stats))
    if missing:
        raise SystemExit(f"no kernel-stats duration for {missing} in {sys.argv[2]}")
    rows = []
    for k, disp in sorted(per.items()):
        n = len(disp)
        avg = {c: sum(d.get(c, 0.0) for d in disp.values()) / n for c in CTRS}
        insts = avg["SQ_INSTS_VALU_FMA_F64"] + avg["SQ_INSTS_VALU_MUL_F64"] + avg["SQ_INSTS_VALU_ADD_F64"] + \
            avg["SQ_INSTS_VALU_TRANS_F64"]
        flops_ub = 64.0 * (2 * avg["SQ_INSTS_VALU_FMA_F64"] + avg["SQ_INSTS_VALU_MUL_F64"] +
                           avg["SQ_INSTS_VALU_ADD_F64"] + avg["SQ_INSTS_VALU_TRANS_F64"])
        r = {"config": cfg, "kernel": k, "launches": n, **{c: avg[c] for c in CTRS},
             "fp64_insts": insts, "fp64_flops_upper": flops_ub,
             "valu_busy": avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"] if avg["SQ_WAVE_CYCLES"] else None}
        r["avg_duration_s"], r["total_duration_s"] = stats[k]
        r["stats_file"] = os.path.basename(sys.argv[2])
        r["executed_TFLOPs_upper"] = flops_ub / stats[k][0] / 1e12
        r["executed_frac_upper"] = r["executed_TFLOPs_upper"] / PEAK
        rows.append(r)
    out = os.path.join(ROOT, "gpurun_out", f"pmc_f64_{cfg}.csv")
    keys = sorted({k for r in rows for k in r}, key=lambda x: (x not in ("config", "kernel", "launches"), x))
    with open(out, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=keys)
        w.writeheader()
        w.writerows(rows)
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
