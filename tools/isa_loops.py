"""Diagnostic: instruction mix of the innermost loops of one kernel in a hipcc `-S` listing.

usage: python tools/isa_loops.py LISTING.s KERNEL_SYMBOL_SUBSTRING [TOP]
Prints, for the largest back-edge loops, the instruction count by opcode family.
"""
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*:", l) and name in l)
    en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    labels = {}
    for i in range(st, en):
        m = re.match(r"^(\.LBB\w+):", lines[i])
        if m:
            labels[m.group(1)] = i

    def mix(a, b):
        c, kinds = 0, {}
        for i in range(a, b):
            s = lines[i].strip()
            if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
                continue
            op = s.split()[0]
            c += 1
            parts = op.split("_")
            k = "_".join(parts[:2]) if len(parts) > 1 else op
            kinds[k] = kinds.get(k, 0) + 1
        return c, kinds

    loops = []
    for i in range(st, en):
        m = re.match(r"\s*s_cbranch_\w+\s+(\.LBB\w+)|\s*s_branch\s+(\.LBB\w+)", lines[i])
        if m:
            t = m.group(1) or m.group(2)
            if t in labels and labels[t] < i:
                c, k = mix(labels[t], i)
                loops.append((c, labels[t] + 1, i + 1, k))
    print(lines[st].split(":")[0], "instructions:", mix(st, en)[0])
    for c, a, b, k in sorted(loops, reverse=True)[:top]:
        valu = sum(v for kk, v in k.items() if kk.startswith("v_"))
        print(f"lines {a}-{b}: {c} instrs, {valu} VALU;",
              ", ".join(f"{kk} {v}" for kk, v in sorted(k.items(), key=lambda x: -x[1])[:12]))


if __name__ == "__main__":
    main()
