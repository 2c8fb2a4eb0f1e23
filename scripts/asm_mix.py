"""Instruction mix of one kernel in a gfx950 .s file: whole body, and each loop (a label that a
later s_cbranch jumps back to). Diagnostic for the VALU/MFMA issue budget.
Usage: python scripts/asm_mix.py file.s kernel_symbol"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_rcp", "v_log", "v_sqrt", "v_rsq", "v_sin", "v_cos")):
        return "trans"
    if op.startswith(("v_mad_u64", "v_mad_i64", "v_mul_hi", "v_mul_lo_u32", "v_mad_u32")):
        return "valu64mul"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "ds"
    if op.startswith(("buffer_", "global_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def body(lines, sym):
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    return lines[start:end]


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    b = body(lines, sym)
    ins = []
    labels = {}
    for i, l in enumerate(b):
        s = l.strip()
        if re.match(r"^\.?L?[\w.]+:", s) and not s.startswith(";"):
            labels[s.split(":")[0]] = len(ins)
            continue
        if not s or s.startswith((";", ".")):
            continue
        ins.append(s.split()[0])
    print("whole kernel:", dict(Counter(classify(o) for o in ins)), "n=", len(ins))
    # loops: backward branches
    for i, l in enumerate(b):
        s = l.strip()
        m = re.match(r"^s_cbranch_\w+\s+(\S+)|^s_branch\s+(\S+)", s)
        if not m:
            continue
        tgt = m.group(1) or m.group(2)
        if tgt in labels:
            # index of this branch in ins
            idx = sum(1 for x in b[:i] if x.strip() and not x.strip().startswith((";", ".")) and not re.match(r"^\.?L?[\w.]+:", x.strip()))
            if labels[tgt] < idx:
                seg = ins[labels[tgt]:idx + 1]
                c = Counter(classify(o) for o in seg)
                print(f"loop {tgt}: {len(seg)} instr", dict(c))
                if len(sys.argv) > 3:
                    print(Counter(o for o in seg if classify(o) == sys.argv[3]).most_common(40))


if __name__ == "__main__":
    main()
