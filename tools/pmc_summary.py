"""Summarise rocprofv3 --pmc CSVs (tools/profile_pmc.sh) per kernel: mean counter value per dispatch.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half of the bytes of a wide
coalesced stream, so HBM read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for 16-B
stores (bytes = WRITE_SIZE * 1024).
Usage: python tools/pmc_summary.py gpurun_out/pmc [out.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(root):
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name") or row.get("Kernel-Name") or row.get("KernelName")
            c = row.get("Counter_Name") or row.get("Counter-Name")
            v = float(row.get("Counter_Value") or row.get("Counter-Value") or 0)
            d = row.get("Dispatch_Id") or row.get("Dispatch-Id")
            per[k][c].append((d, v))
    out = {}
    for k, cs in per.items():
        ent = {}
        for c, vals in cs.items():
            # sum over dimension instances per dispatch, then mean over dispatches
            byd = defaultdict(float)
            for d, v in vals:
                byd[d] += v
            ent[c] = sum(byd.values()) / max(1, len(byd))
        if "FETCH_SIZE" in ent:
            ent["hbm_read_bytes"] = 2 * ent["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in ent:
            ent["hbm_write_bytes"] = ent["WRITE_SIZE"] * 1024
        out[k] = ent
    return out


if __name__ == "__main__":
    res = load(sys.argv[1])
    txt = json.dumps(res, indent=1, sort_keys=True)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt)
    print(txt)
