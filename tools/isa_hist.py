"""Instruction histogram per kernel of a gfx950 assembly file (hipcc --cuda-device-only -S).

    python tools/isa_hist.py k.s [top]

Static counts only (straight-line code dominates the NTT kernels, so static ~ dynamic per thread).
"""
import collections
import re
import sys


def main() -> None:
    lines = open(sys.argv[1]).read().splitlines()
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    name, c = None, collections.Counter()
    for line in lines:
        m = re.match(r"^(_Z\w+):", line)
        if m:
            name, c = m.group(1), collections.Counter()
            continue
        if name is None:
            continue
        t = line.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c[op] += 1
        if op == "s_endpgm":
            tot = sum(c.values())
            valu = sum(v for k, v in c.items() if k.startswith("v_"))
            print(f"{name[:90]}  total {tot}  valu {valu}")
            for k, v in c.most_common(top):
                print(f"   {v:6d} {k}")
            name = None


if __name__ == "__main__":
    main()
