"""How often a kernel's v_mad_u64_u32 waits on the instruction right before it (VERDICT r04 item 3:
do the pass kernels interleave independent MAD chains?).

    python tools/isa_chains.py k.s KERNEL_SUBSTRING [--json out.json]

(k.s: hipcc --cuda-device-only -S of a translation unit.)  For every v_mad_u64_u32 of the first
kernel whose symbol contains KERNEL_SUBSTRING: does its accumulator operand (src2) read the register
pair the previous instruction wrote (distance 1), the one before that (distance 2), or neither?
Also counts the s_nop pads.  A single dependent chain per product shows ~93 % at distance 1.
"""
from __future__ import annotations

import argparse
import json
import re


def kernel_body(text: str, sub: str):
    for m in re.finditer(r"^(_Z\S+):", text, re.M):
        if sub in m.group(1):
            end = text.index(".Lfunc_end", m.end())
            return m.group(1), text[m.end():end]
    raise SystemExit(f"no kernel matching {sub}")


def instructions(body: str):
    out = []
    for line in body.splitlines():
        if not line.startswith("\t"):
            continue
        s = line.strip()
        if not s or s.startswith((".", ";")):
            continue
        out.append(s.split(";")[0].strip())
    return out


def dst(ins: str):
    p = re.split(r"[ ,]+", ins)
    return p[1] if len(p) > 1 else None


def analyse(ins):
    mads = [k for k, s in enumerate(ins) if s.startswith("v_mad_u64_u32")]
    d1 = d2 = 0
    for k in mads:
        acc = re.split(r"[ ,]+", ins[k])[-1]
        if k >= 1 and dst(ins[k - 1]) == acc:
            d1 += 1
        elif k >= 2 and dst(ins[k - 2]) == acc:
            d2 += 1
    n = max(1, len(mads))
    return {"instructions": len(ins), "v_mad_u64_u32": len(mads), "acc_from_previous": d1,
            "acc_from_previous_frac": round(d1 / n, 4), "acc_from_distance_2": d2,
            "acc_from_distance_2_frac": round(d2 / n, 4),
            "s_nop": sum(1 for s in ins if s.startswith("s_nop"))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    name, body = kernel_body(open(a.asm).read(), a.kernel)
    r = {"kernel": name, **analyse(instructions(body))}
    print(json.dumps(r))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(r, fh, indent=1)


if __name__ == "__main__":
    main()
