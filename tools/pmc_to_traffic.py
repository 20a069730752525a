"""Turn rocprofv3 --pmc CSVs (tools/profile_pmc.sh) into per-launch HBM traffic for bench.py.

For the bench's NTT step, the kernel launches of one transform repeat in a fixed order (column
passes, then the final pass).  Per-dispatch HBM bytes = 2 * FETCH_SIZE * 1024 (gfx950 reports half
of a wide coalesced stream, MI355X_MICROARCH.md §HBM) + WRITE_SIZE * 1024, taken from the separate
fetch and write passes and matched by dispatch order.  Writes profiles/pmc_summary.json:
    {tag: {"launch_bytes": [bytes of launch 0, launch 1, ...], "launch_labels": [label of launch 0, ...],
           "launch_kernels": [kernel name of launch 0, ...], "src_hash": H, "profile": DIR}}
(labels as the plan's ntt_plan_last_launch_labels: bench.py attaches the bytes only when its own
launches carry the same labels in the same order)
where H = ntt_amd.build.source_hash() of the tree that was profiled (bench.py reports the bytes only
while the kernel sources still hash to H).
Usage: python tools/pmc_to_traffic.py gpurun_out/pmc TAG [profiles/pmc_summary.json] [--per K] [--note TEXT]
--per K: K launches per step (the four-step's rank-local rows + columns, tools/pmc_ranklocal.sh),
instead of the tail heuristic; --note: stored with the entry (what the bytes cover).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def template_args(name: str, kernel: str):
    """top-level template arguments of `kernel<...>` in a demangled kernel name"""
    i = name.find(kernel + "<")
    if i < 0:
        return None
    i += len(kernel) + 1
    args, depth, cur = [], 0, ""
    while i < len(name):
        ch = name[i]
        if ch == "<":
            depth += 1
        elif ch == ">":
            if depth == 0:
                args.append(cur.strip())
                return args
            depth -= 1
        if ch == "," and depth == 0:
            args.append(cur.strip())
            cur = ""
        else:
            cur += ch
        i += 1
    return None


def launch_label(name: str) -> str:
    """The plan's launch label (include/ntt.h ntt_plan_last_launch_labels) of a kernel name: c<r>[s]
    column pass (s: Shoup-pair outer table), f<r> final, s<r> one transform per workgroup, r<r> several,
    i<r> in-place final with the digit reversal, d digit-reversal swap, b single launch; "" otherwise."""
    a = template_args(name, "k_pass")
    if a and len(a) >= 3:
        kind = {"0": "c", "1": "f", "2": "s", "5": "r"}.get(a[2], "")
        if not kind:
            return ""
        shoup = kind == "c" and len(a) >= 9 and a[8] == "true"
        return f"{kind}{a[1]}" + ("s" if shoup else "")
    a = template_args(name, "k_final_ipn")
    if a and len(a) >= 2:
        return f"i{a[1]}"
    if "k_digitrev_swap" in name:
        return "d"
    if "k_fused" in name:
        return "b"
    return ""


LAUNCH_KERNELS = ("k_pass", "k_final_ipn", "k_digitrev_swap", "k_fused")


def per_dispatch(root, counter):
    rows = defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if (row.get("Counter_Name") or row.get("Counter-Name")) != counter:
                continue
            d = int(row.get("Dispatch_Id") or row.get("Dispatch-Id"))
            rows[d] += float(row.get("Counter_Value") or row.get("Counter-Value") or 0)
            names[d] = row.get("Kernel_Name") or row.get("Kernel-Name")
    return [(names[d], rows[d]) for d in sorted(rows)]


def main():
    argv = list(sys.argv[1:])
    per_arg, note = None, None
    if "--per" in argv:
        i = argv.index("--per")
        per_arg = int(argv[i + 1])
        del argv[i:i + 2]
    if "--note" in argv:
        i = argv.index("--note")
        note = argv[i + 1]
        del argv[i:i + 2]
    root, tag = argv[0], argv[1]
    out = argv[2] if len(argv) > 2 else "profiles/pmc_summary.json"
    fetch = [(k, v) for k, v in per_dispatch(os.path.join(root, "fetch"), "FETCH_SIZE")
             if any(x in k for x in LAUNCH_KERNELS)]
    write = [(k, v) for k, v in per_dispatch(os.path.join(root, "write"), "WRITE_SIZE")
             if any(x in k for x in LAUNCH_KERNELS)]
    # launches per transform = number of distinct consecutive pass kernels at the tail
    names = [k for k, _ in fetch]
    per = 1
    while per < len(names) and not ("KIND_FINAL" in names[per - 1] or ", 1, " in names[per - 1]):
        per += 1
    if per_arg:
        per = per_arg
    steps = len(fetch) // per
    traffic = []
    for i in range(per):
        f = [fetch[s * per + i][1] for s in range(1, steps)] or [fetch[i][1]]
        w = [write[s * per + i][1] for s in range(1, steps)] or [write[i][1]]
        traffic.append(2 * 1024 * sum(f) / len(f) + 1024 * sum(w) / len(w))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from ntt_amd.build import source_hash
    d = json.load(open(out)) if os.path.exists(out) else {}
    labels = [launch_label(fetch[i][0]) for i in range(per)]
    assert labels == [launch_label(write[i][0]) for i in range(per)], "fetch and write passes differ"
    d[tag] = {"launch_bytes": traffic, "launch_labels": labels, "launch_kernels": [fetch[i][0] for i in range(per)],
              "src_hash": source_hash(), "profile": root}
    if note:
        d[tag]["note"] = note
    json.dump(d, open(out, "w"), indent=1)
    print(tag, [f"{lab}: {t / 1e9:.3f} GB" for lab, t in zip(labels, traffic)])


if __name__ == "__main__":
    main()
