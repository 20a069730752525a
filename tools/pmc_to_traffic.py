"""Turn rocprofv3 --pmc CSVs (tools/profile_pmc.sh) into per-launch HBM traffic for bench.py.

For the bench's NTT step, the kernel launches of one transform repeat in a fixed order (column
passes, then the final pass).  Per-dispatch HBM bytes = 2 * FETCH_SIZE * 1024 (gfx950 reports half
of a wide coalesced stream, MI355X_MICROARCH.md §HBM) + WRITE_SIZE * 1024, taken from the separate
fetch and write passes and matched by dispatch order.  Writes profiles/pmc_summary.json:
    {tag: {"launch_bytes": [bytes of launch 0, launch 1, ...], "src_hash": H, "profile": DIR}}
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
    fetch = [(k, v) for k, v in per_dispatch(os.path.join(root, "fetch"), "FETCH_SIZE") if "k_pass" in k]
    write = [(k, v) for k, v in per_dispatch(os.path.join(root, "write"), "WRITE_SIZE") if "k_pass" in k]
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
    d[tag] = {"launch_bytes": traffic, "src_hash": source_hash(), "profile": root}
    if note:
        d[tag]["note"] = note
    json.dump(d, open(out, "w"), indent=1)
    print(tag, [f"{t / 1e9:.3f} GB" for t in traffic])


if __name__ == "__main__":
    main()
