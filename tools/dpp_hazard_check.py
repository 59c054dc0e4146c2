"""Static check of the VALU-write -> DPP-read hazard in a gfx950 assembly listing (hipcc -S).

A DPP instruction whose broadcast source VGPR was written by a VALU instruction fewer than 2 instructions
earlier reads a stale value (2 wait states are required; s_nop N provides N + 1).  The inline-asm recursions
of mpcqp.hip are outside the compiler's hazard recognizer, so they pad by hand; this script checks every
v_*_dpp of a listing (straight-line look-back within a basic block; a label resets the window).

  python tools/dpp_hazard_check.py listing.s [kernel-name-substring]"""
import re
import sys

VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(tok):
    out = set()
    for m in VREG.finditer(tok):
        if m.group(1):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def check(lines):
    bad = []
    window = []          # recent (wait_states, written regs) entries, newest last
    for no, raw in lines:
        line = raw.split(";")[0].strip()
        if not line or line.startswith("."):
            continue
        if re.match(r"^[\w.$]+:", line):
            window = []
            continue
        op = line.split()[0]
        args = line[len(op):].strip()
        if "_dpp" in op and op.startswith("v_"):
            ops = [a.strip() for a in args.split(",")]
            src = regs(ops[1]) if len(ops) > 1 else set()
            dist = 0
            for ws, wr in reversed(window):
                if dist >= 2:
                    break
                if wr & src:
                    bad.append((no, raw.strip(), dist))
                    break
                dist += ws
        if op == "s_nop":
            ws = int(args, 0) + 1 if args else 1
            window.append((ws, set()))
        else:
            written = set()
            if op.startswith("v_") and not op.startswith("v_cmp") and not op.startswith("v_readlane") \
                    and not op.startswith("v_readfirstlane"):
                first = args.split(",")[0]
                written = regs(first)
            window.append((1, written))
        window = window[-4:]
    return bad


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else None
    src = open(path).read().split("\n")
    funcs, cur, name = [], [], None
    for i, l in enumerate(src):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            if name:
                funcs.append((name, cur))
            name, cur = m.group(1), []
            continue
        if name and l.startswith(".Lfunc_end"):
            funcs.append((name, cur))
            name, cur = None, []
            continue
        if name:
            cur.append((i + 1, l))
    total = 0
    for name, body in funcs:
        if want and want not in name:
            continue
        b = check(body)
        ndpp = sum(1 for _, l in body if "_dpp" in l.split(";")[0])
        print(f"{name[:70]}: {ndpp} DPP instructions, {len(b)} hazards")
        for no, text, dist in b[:10]:
            print(f"   line {no}: {text}  (source written {dist} wait states before)")
        total += len(b)
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
