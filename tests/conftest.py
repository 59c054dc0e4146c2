"""Shared pytest setup.

Markers:  gpu — needs a real MI355X (run with `-m gpu` on the GPU box).
The package directory name (safe-autonomous-driving-mpc_amd) is not an importable Python
identifier, so — exactly like the reference's flat scripts — its modules are imported by
putting the directory on sys.path (`import trajectory_tracking`, `import mpcqp`, ...).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "safe-autonomous-driving-mpc_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP device)")


def pytest_collection_finish(session):
    """GPU runs: load torch's HIP runtime before libmpcqp.so is loaded.  Both carry the soname
    libamdhip64.so.7; whichever loads first serves the process, and torch cannot initialise on the
    system runtime that libmpcqp would pull in (bench.py imports torch first for the same reason).
    libmpcqp itself works on either."""
    if any(item.get_closest_marker("gpu") for item in session.items):
        try:
            import torch
            torch.cuda.is_available()
        except ImportError:
            pass


def load_golden(name):
    """Load tests/golden/<name>.npz (allow_pickle=False) into a dict of arrays."""
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_cases(name):
    g = load_golden(name)
    n = int(g["n"])
    out = []
    for j in range(n):
        pre = f"c{j}_"
        out.append({k[len(pre):]: v for k, v in g.items() if k.startswith(pre)})
    return out, g


def traj_arrays(i):
    with np.load(os.path.join(PKG, "data", f"trajectory{i}.npz"), allow_pickle=False) as z:
        return z["X"], z["U"]


@pytest.fixture(scope="session")
def oracles():
    import oracle as O
    O.build()
    return {i: O.Oracle(*traj_arrays(i)) for i in (1, 2, 3)}
