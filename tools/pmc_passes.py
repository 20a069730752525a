"""Per-pass view of rocprofv3 --pmc runs (tools/r06.sh pmc24): for every k_pass / fused kernel, the
mean over dispatches of each counter, the kernel's duration in the SAME run (its counter-collection
timestamps), and the derived figures: GRBM_GUI_ACTIVE / 8 XCDs = cycles, cycles / duration = clock,
VALU instructions per wave, LDS bank-conflict cycles per LDS instruction, HBM bytes (FETCH_SIZE x 2
per MI355X_MICROARCH.md, WRITE_SIZE exact).

    python tools/pmc_passes.py gpurun_out/r06_a/pmc_tp [--json out.json]
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.match(r"void ntt::(\w+)<ntt::Eng29<([\d, ]+)>, (\d+), (\d+)((?:, \w+)*)>", name)
    if m:
        kind = {"0": "col", "1": "fin", "2": "single", "5": "rows"}.get(m[4], m[4])
        shoup = kind == "col" and m[5].split(", ")[-1] == "true"  # SHTW: Shoup-pair outer table (pass >= 2)
        return f"{m[1]}<{m[2].replace(' ', '')}>:r{m[3]}:{kind}" + (":shoup" if shoup else "")
    m = re.match(r"void ntt::(\w+)", name)
    return m[1] if m else name[:40]


def load(root: str):
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> sum
    dur = defaultdict(dict)  # kernel -> dispatch -> ns
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        grp = os.path.relpath(f, root).split(os.sep)[0]
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            d = (grp, row["Dispatch_Id"])
            per[k][row["Counter_Name"]][d] += float(row["Counter_Value"])
            if "GRBM_GUI_ACTIVE" == row["Counter_Name"]:
                dur[k][d] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    out = {}
    for k, cs in per.items():
        e = {c: sum(v.values()) / len(v) for c, v in cs.items()}
        if dur[k]:
            e["duration_us"] = sum(dur[k].values()) / len(dur[k]) / 1e3
        if "GRBM_GUI_ACTIVE" in e:
            e["cycles"] = e["GRBM_GUI_ACTIVE"] / 8
            if "duration_us" in e:
                e["clock_ghz"] = e["cycles"] / (e["duration_us"] * 1e3)
        if "SQ_INSTS_VALU" in e and e.get("SQ_WAVES"):
            e["valu_per_wave"] = e["SQ_INSTS_VALU"] / e["SQ_WAVES"]
        if "SQ_LDS_BANK_CONFLICT" in e and e.get("SQ_INSTS_LDS"):
            e["lds_conflict_per_inst"] = e["SQ_LDS_BANK_CONFLICT"] / e["SQ_INSTS_LDS"]
        if "FETCH_SIZE" in e:
            e["hbm_read_GB"] = 2 * e["FETCH_SIZE"] * 1024 / 1e9
        if "WRITE_SIZE" in e:
            e["hbm_write_GB"] = e["WRITE_SIZE"] * 1024 / 1e9
        if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e:
            e["l2_hit"] = e["TCC_HIT_sum"] / max(1.0, e["TCC_HIT_sum"] + e["TCC_MISS_sum"])
        out[k] = e
    return out


def main():
    root = sys.argv[1]
    res = load(root)
    keys = ["duration_us", "cycles", "clock_ghz", "valu_per_wave", "SQ_WAVES", "lds_conflict_per_inst",
            "SQ_INSTS_LDS", "hbm_read_GB", "hbm_write_GB", "l2_hit"]
    for k in sorted(res):
        if not any(s in k for s in ("k_pass", "k_fused", "k_final")):
            continue
        e = res[k]
        print(k, " ".join(f"{x}={e[x]:.4g}" for x in keys if x in e))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as fh:
            json.dump(res, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
