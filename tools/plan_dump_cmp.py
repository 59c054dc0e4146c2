"""Bit-for-bit comparison of tools/plan_probe.py dumps (PLAN_DUMP=1) of two planner library variants.
usage: python tools/plan_dump_cmp.py libA.so libB.so N B"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
a, b, N, B = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
da = np.load(os.path.join(ROOT, "gpurun_out", f"plan_dump_{a}_{N}_{B}.npz"))
db = np.load(os.path.join(ROOT, "gpurun_out", f"plan_dump_{b}_{N}_{B}.npz"))
same = {k: bool(np.array_equal(da[k], db[k])) for k in da.files}
print(f"{a} vs {b} N={N} B={B}: " + ", ".join(f"{k} {'identical' if v else 'DIFFERENT'}" for k, v in same.items()))
if not all(same.values()):
    d = np.abs(da["X"] - db["X"]).reshape(int(B), -1).max(axis=1)
    print(f"  chunks differing: {int((d > 0).sum())}, max |dX| {d.max():.3e}; status agree "
          f"{float((da['status'] == db['status']).mean()):.4f}")
