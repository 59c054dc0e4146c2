"""Summarise rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of the solver kernel into
profiles/pmc_hbm_bytes.json: HBM bytes per launch, with the gfx950 corrections of
MI355X_MICROARCH.md (FETCH_SIZE is in KiB and counts half the bytes of wide coalesced reads)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, counter):
    """Counter value per solver dispatch (dict dispatch id -> (kernel name, value))."""
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "mpc_solve_kernel" not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            k = row.get("Dispatch_Id") or row.get("Correlation_Id")
            name, v = vals.get(k, (row["Kernel_Name"], 0.0))
            vals[k] = (name, v + float(row["Counter_Value"]))
    return vals


def per_step(vals):
    """Bytes per bench step: a step is one MODE_FULL launch, or a MODE_XO + MODE_IPM pair (the
    two-phase launch); the template's third argument is the mode."""
    steps = sum(1 for name, _ in vals.values() if ", 1, " not in name.split("<", 1)[1].split(">")[0] + ", ")
    return sum(v for _, v in vals.values()) / max(1, steps), steps


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
    round_tag = sys.argv[2] if len(sys.argv) > 2 else None
    commit = sys.argv[3] if len(sys.argv) > 3 else None
    fetch = per_dispatch(os.path.join(ROOT, "gpurun_out", "pmc_fetch"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(ROOT, "gpurun_out", "pmc_write"), "WRITE_SIZE")
    if not fetch or not write:
        raise SystemExit(f"no counter rows found (fetch {len(fetch)}, write {len(write)})")
    f_kib, nf = per_step(fetch)
    w_kib, nw = per_step(write)
    out_path = os.path.join(ROOT, "profiles", "pmc_hbm_bytes.json")
    res = json.load(open(out_path)) if os.path.exists(out_path) else {}
    # FETCH_SIZE x 2 (gfx950: 128-B requests tallied at 64 B), KiB -> bytes
    res[cfg] = 2.0 * f_kib * 1024.0 + w_kib * 1024.0
    res[cfg + "_detail"] = {"FETCH_SIZE_KiB_per_step": f_kib, "WRITE_SIZE_KiB_per_step": w_kib,
                            "dispatches": [len(fetch), len(write)], "steps": [nf, nw],
                            "bytes_per_step": res[cfg],
                            "correction": "traffic = 2*FETCH_SIZE + WRITE_SIZE (KiB->B); MI355X_MICROARCH HBM section",
                            "round": round_tag, "commit": commit}
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res[cfg + "_detail"]))


if __name__ == "__main__":
    main()
