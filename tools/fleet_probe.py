"""Fleet leg breakdown (bench.plan_fleet): the device chunk loop's launches, the host assembly and checks;
with the plans dispatched longest remaining distance first, then in index order for comparison.
usage: python tools/fleet_probe.py [B]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "safe-autonomous-driving-mpc_amd"), ROOT]
import torch  # noqa: E402

torch.cuda.init()       # torch's HIP runtime before the planner's (the two HIP runtimes)
import bench  # noqa: E402
import mpcplan  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
import numpy as np  # noqa: E402
for label in ("longest first", "index order"):
    if label == "index order":
        _argsort = np.argsort
        np.argsort = lambda a, kind=None: _argsort(np.zeros_like(a), kind="stable")
    f = bench.plan_fleet(B, 0)
    print(label, json.dumps({k: f[k] for k in ("seconds", "chunks", "checks_passed", "breakdown")}), flush=True)
