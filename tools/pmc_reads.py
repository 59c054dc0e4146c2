"""Summary of tools/gpu/pmc_reads.sh: per-dispatch counter means of the C2 solver kernels (crossover
MODE_XO, interior point MODE_IPM) for each pass, and a linear fit over B of FETCH_SIZE per kernel (per-launch
intercept vs per-instance slope).  Writes profiles/r05_pmc_reads.csv and prints a table, then the attribution: each kernel's code-object
size (C2: MODE_IPM / MODE_XO instantiation at N = 20 without obstacles) times the 8 XCDs, whose L2s each
fetch the code once per launch, against the per-launch intercept."""
import csv
import glob
import os
import re

import subprocess
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def mode(name):
    m = re.search(r"mpc_solve_kernel<(\d+), (\w+), (\d+), (\d+)>", name) or \
        re.search(r"mpc_solve_kernelILi(\d+)ELb([01])ELi(\d+)ELi(\d+)E", name)
    if not m:
        return None
    return {"1": "XO", "2": "IPM", "0": "FULL", "3": "ONE"}[m.group(3)]


def pass_means(tag):
    """{(kernel mode, counter): mean per dispatch} over the pass's solver dispatches (warm-up included)."""
    acc = {}
    for f in glob.glob(os.path.join(OUT, f"pmcr_{tag}", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            md = mode(row.get("Kernel_Name", ""))
            if md is None:
                continue
            key = (md, row["Counter_Name"], row.get("Dispatch_Id") or row.get("Correlation_Id"))
            acc[key] = acc.get(key, 0.0) + float(row["Counter_Value"])
    res = {}
    for (md, cn, _), v in acc.items():
        res.setdefault((md, cn), []).append(v)
    return {k: (float(np.mean(v)), len(v)) for k, v in res.items()}


def code_sizes(so_path):
    """{mode: bytes} of the C2 kernels (mpc_solve_kernel<32, false, mode, 20>) in the library's gfx950 code object"""
    llvm = "/opt/rocm/lib/llvm/bin"
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fatbin"), os.path.join(d, "dev.co")
        subprocess.run([f"{llvm}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", so_path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        syms = subprocess.run([f"{llvm}/llvm-readelf", "-s", "--wide", co], check=True, capture_output=True,
                              text=True).stdout
    out = {}
    for line in syms.splitlines():
        f = line.split()
        if len(f) >= 8 and f[3] == "FUNC":
            m = re.search(r"mpc_solve_kernelILi32ELb0ELi(\d)ELi20E", f[7])
            if m:
                out[{"1": "XO", "2": "IPM"}.get(m.group(1), m.group(1))] = int(f[2])
    return out


def main():
    rows = []
    fits = {}
    for tag in ["fetch_1024", "fetch_2048", "fetch_4096", "tcc_1024", "tcc_2048", "tcc_4096", "tcp_1024", "tcp_2048",
                "tcp_4096", "fetch_dbg"]:
        m = pass_means(tag)
        B = 4096 if tag.endswith("dbg") else int(tag.split("_")[1])
        for (md, cn), (v, n) in sorted(m.items()):
            rows.append({"pass": tag, "batch": B, "kernel": md, "counter": cn, "mean_per_dispatch": v, "dispatches": n})
            if tag.startswith("fetch_") and not tag.endswith("dbg"):
                fits.setdefault(md, []).append((B, v))
    path = os.path.join(ROOT, "profiles", "r05_pmc_reads.csv")
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()) if rows else ["pass"])
        w.writeheader()
        w.writerows(rows)
    for r in rows:
        print(f"{r['pass']:11s} B={r['batch']:5d} {r['kernel']:4s} {r['counter']:28s} {r['mean_per_dispatch']:14.1f} "
              f"({r['dispatches']} dispatches)")
    for md, pts in fits.items():
        b = np.array([p[0] for p in pts], float)
        v = np.array([p[1] for p in pts], float)
        if len(b) >= 2:
            slope, icpt = np.polyfit(b, v, 1)
            print(f"FETCH_SIZE fit {md}: {icpt:.1f} KiB per launch + {slope * 1024:.1f} B per instance "
                  f"(KiB as counted; x2 for 128-B requests tallied at 64 B)")
    so = os.path.join(ROOT, "safe-autonomous-driving-mpc_amd", "libmpcqp.so")
    if os.path.exists(so):
        cs = code_sizes(so)
        tot = {md: dict(pts)[4096] for md, pts in fits.items() if 4096 in dict(pts)}
        code = {md: 8 * cs.get(md, 0) / 1024 for md in tot}
        for md in tot:
            print(f"{md}: code object {cs.get(md, 0)} B x 8 XCDs = {code[md]:.0f} KiB of {tot[md]:.0f} KiB counted at "
                  f"B = 4096 ({code[md] / tot[md] * 100:.0f}%)")
        print(f"both kernels: code {sum(code.values()):.0f} KiB of {sum(tot.values()):.0f} KiB counted "
              f"({sum(code.values()) / sum(tot.values()) * 100:.0f}%)")


if __name__ == "__main__":
    main()
