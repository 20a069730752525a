"""Stress of the inter-workgroup hand-offs (k_final_ipn: the in-place plans' fused digit reversal;
k_fused3 / k_fused3b / k_fused2b / k_fused2bi: NTT_PLAN_SINGLE_LAUNCH): many transforms of fresh random vectors through each, every output
compared with the default schedule's and the watchdog status checked, so that a rare ordering race
would show as a mismatch.

    python tools/stress_sync.py [--reps 40] [--out gpurun_out/stress.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# flags joined by '+' (round 5: the two-pass single launch at 2^20, k_fused2b, and its in-place form
# k_fused2bi; BLS12-381 too)
CASES = [(1, 20, 4, "in_place"), (1, 24, 4, "in_place"), (0, 22, 1, "in_place"), (0, 26, 1, "in_place"),
         (2, 22, 4, "in_place"), (1, 18, 4, "single_launch"), (1, 20, 4, "single_launch"),
         (2, 22, 4, "single_launch"), (1, 20, 4, "in_place+single_launch"), (2, 20, 4, "single_launch"),
         (2, 20, 4, "in_place+single_launch"), (1, 19, 4, "in_place+single_launch")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch
    from ntt_amd.ntt import NTTPlan
    rows = []
    for fid, lg, limbs, flag in CASES:
        ref = NTTPlan(fid, lg, limbs)
        pl = NTTPlan(fid, lg, limbs, **{f: True for f in flag.split("+")})
        bad = 0
        t0 = time.perf_counter()
        for rep in range(a.reps):
            x = ref.fill(ref.empty(), "random", seed=1000 + rep)
            y = x.clone()
            ref.forward(x)
            pl.forward(y)
            inv = rep % 2 == 1  # alternate directions: the inverse's hand-offs too
            if inv:
                ref.inverse(x)
                pl.inverse(y)
            if not torch.equal(x, y):
                bad += 1
        st = pl.device_status()
        r = {"field": fid, "log_n": lg, "limbs64": limbs, "schedule": flag, "reps": a.reps, "mismatches": bad,
             "device_status": st, "seconds": round(time.perf_counter() - t0, 2)}
        rows.append(r)
        print(json.dumps(r), flush=True)
        del ref, pl
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")
    if any(r["mismatches"] or r["device_status"] for r in rows):
        sys.exit(1)


if __name__ == "__main__":
    main()
