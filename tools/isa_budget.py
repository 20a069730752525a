"""Per-category VALU instruction budget of one kernel from a gfx950 assembly file with line tables
(hipcc --cuda-device-only -S -gline-tables-only ...).

    python tools/isa_budget.py k.s KERNEL_SUBSTRING [--elems-per-thread 4] [--json out.json]

Every instruction is attributed to the innermost source location of its `.loc` directive, that
location to the enclosing function of the source file (a function starts at a line that opens a
`__device__` / `__global__` definition and runs to the next one), and the function to a category
(CATEGORIES below).  Counts are static (per thread, both sides of the two wave-uniform branches
included); divided by the elements per thread they are a per-element budget.  v_mad_u64_u32 is
counted separately inside every category.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re

# function name -> category (first match wins; unlisted functions of a file fall to FILE_DEFAULT)
CATEGORIES = [
    (r"^mulc29", "Shoup product (mulc29: twiddle x element)"),
    (r"^mont29", "Montgomery product (mont29: outer twiddle / variable x variable)"),
    (r"^(bfly_raw|bfly_raw_w|bfly_lk|bfly_l|bfly_w_l|dft_q_fast|dft_q|dft)$", "butterfly add/sub (+ padded K p offsets)"),
    (r"^(norm_u|norm_s|norm)$", "carry normalisation (norm_u / norm_s)"),
    (r"^(reduce_top|reduce|reduce_chain|cond_sub|cond_sub_rare|store_lazy|store)$", "reductions (quotient estimate, conditional subtractions)"),
    (r"^(pack29|unpack29|load|put|store_wt16)$", "HBM format: pack29 / unpack29 + vector loads/stores"),
    (r"^(tload|twiddle_mul|twiddle_mul_lds|mul|mul_u|mulv)$", "twiddle-table loads and product call glue"),
    (r"^(lds_put_part|lds_get_part|lds_slot)$", "LDS exchange (slot addressing, ds_read/ds_write)"),
    (r"^(substage|sub_map|natural_index|pass_tile|k_pass|brev_bits|static_for|static_for_impl|operator\(\))$",
     "tile addressing and control (positions, group maps, branches)"),
]
FILE_DEFAULT = {
    "field29_asm9.hpp": "Shoup product (mulc29: twiddle x element)",
    "field29.hpp": "carry normalisation (norm_u / norm_s)",
}
FUNC_RE = re.compile(r"(__device__|__global__|__host__ __device__|F29_HD)[^;{]*?\b(\w+)\s*\(")


def function_map(path: str):
    """[(start_line, name)] for one source file (1-based lines)."""
    out = []
    lines = open(path).read().splitlines()
    for i, line in enumerate(lines, 1):
        m = FUNC_RE.search(line)
        if m and not line.strip().startswith("//"):
            out.append((i, m.group(2)))
        elif re.match(r"^\s*(auto|const auto)\s+\w+\s*=\s*\[", line):  # lambdas inside kernels
            out.append((i, "operator()"))
    return out


def category(fname: str, func: str) -> str:
    for pat, cat in CATEGORIES:
        if re.search(pat, func):
            return cat
    return FILE_DEFAULT.get(fname, f"other ({fname}:{func})")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--elems-per-thread", type=int, default=4)
    ap.add_argument("--json", default="")
    ap.add_argument("--by-func", action="store_true", help="also list the source functions")
    a = ap.parse_args()
    files, fmaps = {}, {}
    cur = None
    in_k = False
    valu = collections.Counter()
    mads = collections.Counter()
    other = collections.Counter()
    ops = collections.Counter()
    byf, byf_mad = collections.Counter(), collections.Counter()
    name = None
    for line in open(a.asm):
        t = line.strip()
        m = re.match(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', t)
        if m:
            d, f = m.group(2), m.group(3)
            files[int(m.group(1))] = os.path.join(d, f) if f else d
            continue
        m = re.match(r"^(_Z\w+):", line)
        if m:
            in_k = a.kernel in m.group(1) and name is None
            if in_k:
                name = m.group(1)
            continue
        if not in_k:
            continue
        if t.startswith(".Lfunc_end"):  # the kernel's end (s_endpgm may also appear on early-exit paths)
            in_k = False
            continue
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            cur = (int(m.group(1)), int(m.group(2)))
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        path = files.get(cur[0], "?") if cur else "?"
        fname = os.path.basename(path)
        if path not in fmaps:
            fmaps[path] = function_map(path) if os.path.exists(path) else []
        func = "?"
        for start, nm in fmaps[path]:
            if start <= cur[1]:
                func = nm
            else:
                break
        cat = category(fname, func)
        if op.startswith("v_"):
            byf[(fname, func)] += 1
            byf_mad[(fname, func)] += op == "v_mad_u64_u32"
            valu[cat] += 1
            ops[op] += 1
            if op == "v_mad_u64_u32":
                mads[cat] += 1
        else:
            other[op.split("_")[0] + "_" + (op.split("_")[1] if "_" in op else "")] += 1
    if name is None:
        raise SystemExit(f"no kernel matching {a.kernel}")
    ept = a.elems_per_thread
    tot = sum(valu.values())
    print(f"{name[:110]}\n  VALU {tot} static per thread = {tot / ept:.0f} per element "
          f"(v_mad_u64_u32 {sum(mads.values()) / ept:.0f} per element)")
    rows = []
    for cat, v in valu.most_common():
        print(f"  {v / ept:7.1f} /elem  {v / tot:6.1%}  (MAD {mads[cat] / ept:6.1f})  {cat}")
        rows.append({"category": cat, "valu_per_elem": v / ept, "mad_per_elem": mads[cat] / ept, "share": v / tot})
    print("  top non-MAD VALU opcodes:", ", ".join(f"{k} {v / ept:.0f}" for k, v in ops.most_common(14)
                                                if k != "v_mad_u64_u32"))
    if a.by_func:
        for k, v in byf.most_common(25):
            print(f"    {v / ept:7.1f} /elem (MAD {byf_mad[k] / ept:6.1f})  {k[0]}:{k[1]}")
    if a.json:
        json.dump({"kernel": name, "valu_static_per_thread": tot, "elems_per_thread": ept, "categories": rows,
                   "opcodes_per_elem": {k: v / ept for k, v in ops.most_common()},
                   "non_valu": dict(other)}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
