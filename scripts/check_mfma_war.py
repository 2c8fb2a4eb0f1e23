"""Static check of a gfx950 .s listing: instructions that WRITE a VGPR which one of the
preceding MFMAs (within a window of issued instructions) reads as its A or B source.
Usage: python scripts/check_mfma_war.py file.s [kernel_substring] [window]"""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    window = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    kernel, hits, recent = None, {}, []
    for line in open(path):
        s = line.split(";")[0].strip()
        if s.endswith(":") and not s.startswith("."):
            kernel, recent = s[:-1], []
            continue
        if not s or s.startswith(";") or s.startswith(".") or kernel is None or want not in kernel:
            continue
        parts = s.replace(",", " ").split()
        op = parts[0]
        if op.startswith("s_") and op not in ("s_nop",):
            continue
        if op == "s_nop":
            recent = recent[int(parts[1]) + 1:] if len(parts) > 1 else recent[1:]
            continue
        dst = regs(parts[1]) if len(parts) > 1 and not op.startswith(("ds_write", "buffer_store", "global_store")) else set()
        for k, (mop, srcs) in enumerate(recent):
            if dst & srcs:
                hits.setdefault(kernel, []).append((len(recent) - k, op, mop))
        if op.startswith("v_mfma"):
            srcs = regs(parts[2]) | regs(parts[3])
            recent.append((op, srcs))
        else:
            recent.append(("", set()))
        recent = recent[-window:]
    import collections
    for k, h in hits.items():
        kinds = collections.Counter((d, op.split("_")[0] + "_" + op.split("_")[1]) for d, op, _ in h)
        print(f"{k[:75]}: {len(h)}: " + ", ".join(f"{op}@{d}:{n}" for (d, op), n in sorted(kinds.items())))


if __name__ == "__main__":
    main()
