"""bench.py's multi-rank launch: `python bench.py --gpus N` without torchrun starts N
rank processes itself, and a rank whose WORLD_SIZE disagrees with --gpus refuses to run.  The ranks use
the `--device cpu` stand-in (libmpcqp's host backend, gloo), the same sharded path as the GPU ranks."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=e, timeout=600)


def test_self_launch_two_ranks():
    r = _run(["--gpus", "2", "--device", "cpu", "--steps", "2", "--warmup", "1", "--batch", "48", "--no-cpu",
              "--closed-loop", "6"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 alone prints the result line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["solver"]["ranks"] == 2 and d["solver"]["egos"] == 96
    assert d["config"]["global_batch"] == 96
    assert d["closed_loop"]["ranks"] == 2 and d["closed_loop"]["egos"] == 12
    assert d["device"] == "cpu-standin"


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "2", "--device", "cpu", "--steps", "1", "--warmup", "0", "--batch", "8", "--no-cpu",
              "--closed-loop", "0"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr
