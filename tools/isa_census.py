"""Static instruction census of one kernel in a hipcc --save-temps .s file (diagnostic).
  python tools/isa_census.py FILE.s SUBSTRING   (SUBSTRING selects the kernel symbol, e.g. ILi32ELb0ELi2ELi20E)"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(_Z16mpc_solve_kernel\w*" + re.escape(sys.argv[2]) + r"\w*):", s, re.M)
i = m.start()
j = s.index(".Lfunc_end", i)
c = collections.Counter()
n = 0
for line in s[i:j].splitlines():
    t = line.strip().split()
    if not t or t[0].startswith((".", ";", "_")) or t[0].endswith(":"):
        continue
    op = t[0]
    n += 1
    if op.startswith(("scratch_", "buffer_")):
        c["scratch " + op] += 1
    elif op.startswith("v_accvgpr"):
        c["accvgpr move"] += 1
    elif op.startswith("ds_"):
        c["lds"] += 1
    elif op.startswith("s_waitcnt") or op.startswith("s_nop"):
        c[op] += 1
    elif op.startswith("s_"):
        c["salu/branch"] += 1
    elif op.startswith("v_") and "f64" in op:
        c["valu f64"] += 1
    elif op.startswith("v_"):
        c["valu other"] += 1
    else:
        c[op] += 1
print(m.group(1)[:60], "static instructions", n)
for k, v in sorted(c.items(), key=lambda x: -x[1]):
    print(f"  {k:28s} {v}")
