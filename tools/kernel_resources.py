"""Per-kernel resources of the built libmpcqp.so, read from the gfx950 code object's metadata notes
(no GPU needed): scratch bytes per lane (.private_segment_fixed_size), VGPRs and AGPRs.

  python tools/kernel_resources.py [path/to/libmpcqp.so]      -> JSON list on stdout

Used by tests/test_kernel_resources.py: the library is built with -Wno-pass-failed, so a full unroll
that silently fails in a horizon-specialised kernel (dynamic indexing of the unrolled records) would
show up here as scratch, not as a warning."""
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_resources(so_path):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fatbin"), os.path.join(d, "dev.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", so_path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out, cur = [], None
    for line in notes.splitlines():
        t = line.strip().lstrip("- ").strip()
        m = re.match(r"\.(name|private_segment_fixed_size|vgpr_count|agpr_count):\s+(\S+)", t)
        if not m:
            continue
        key, val = m.groups()
        if key == "agpr_count":          # first field of each kernel record in the notes
            cur = {"agpr": int(val)}
            out.append(cur)
        elif cur is not None:
            cur[{"name": "name", "private_segment_fixed_size": "scratch", "vgpr_count": "vgpr"}[key]] = (
                val if key == "name" else int(val))
    return [k for k in out if "name" in k]


def solver_kernel_key(name):
    """(GL, OBS, MODE, NT) of a mangled mpc_solve_kernel<GL, OBS, MODE, NT> name, else None."""
    m = re.search(r"mpc_solve_kernelILi(\d+)ELb([01])ELi(\d+)ELi(\d+)E", name)
    return tuple(int(x) for x in m.groups()) if m else None


if __name__ == "__main__":
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "safe-autonomous-driving-mpc_amd", "libmpcqp.so")
    print(json.dumps(kernel_resources(so), indent=1))
