"""Two-sided piece schedules of the four-step on one GPU (VirtualRanks: the exchange = device copies on a
side stream), ms per forward and per inverse for each (world, log_n, row pieces, column pieces).

    python tools/exp_pieces.py [--out gpurun_out/x.jsonl]

On one GPU the copies compete with the transforms for HBM and CUs, so this measures what the pieces cost
(smaller launches, more copy calls) rather than what they hide; the hiding needs a multi-GPU node.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CFGS = [(2, 24, 1, 1), (2, 24, 2, 1), (2, 24, 2, 2), (2, 24, 4, 4), (8, 24, 1, 1), (8, 24, 2, 2),
        (8, 28, 1, 1), (8, 28, 4, 1), (8, 28, 4, 4), (8, 28, 8, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cfg", action="append", default=[], help="world,log_n,row_pieces,col_pieces (repeatable)")
    ap.add_argument("--forward-only", action="store_true")
    ap.add_argument("--extra-streams", type=int, default=0,
                    help="create this many torch streams first (moves the side stream to another hardware queue)")
    a = ap.parse_args()
    cfgs = [tuple(int(v) for v in c.split(",")) for c in a.cfg] or CFGS
    import torch
    from ntt_amd.distributed import VirtualRanks
    keep = [torch.cuda.Stream() for _ in range(a.extra_streams)]
    rows = []
    for world, lg, rp, cp in cfgs:
        vr = VirtualRanks(1, lg, 4, world, pieces=rp, col_pieces=cp)
        xs = vr.fill(vr.empty(), "random", seed=4)
        res = {"world": world, "log_n": lg, "row_pieces": vr.fs.rp, "col_pieces": vr.fs.cp}
        runs = (("forward_ms", vr.forward),) if a.forward_only else (("forward_ms", vr.forward), ("inverse_ms", vr.inverse))
        for name, fn in runs:
            for _ in range(3):
                fn(xs)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                fn(xs)
            torch.cuda.synchronize()
            res[name] = (time.perf_counter() - t0) / a.reps * 1e3
        rows.append(res)
        print(json.dumps(res), flush=True)
        del vr, xs
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
