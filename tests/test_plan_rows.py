"""The planner kernel's row-parallel slot decoding (row_at, csrc/plan_kernel.h) against its per-stage row visit
(for_rows / row_sp) for every horizon 1..64, intermediate and final chunks, every slot: stage, presence,
variables and coefficients bit for bit.  Runs the kernel source on the host through tools/plan_emu.cpp."""
import os
import subprocess

from conftest import ROOT


def test_row_slots_match_the_stage_visit(tmp_path):
    exe = str(tmp_path / "plan_emu")
    subprocess.run(["g++", "-std=c++17", "-O1", os.path.join(ROOT, "tools", "plan_emu.cpp"), "-o", exe, "-lpthread"],
                   check=True, capture_output=True)
    out = subprocess.run([exe, "--rows"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 mismatches" in out.stdout
