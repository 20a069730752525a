"""Per-transform time of batched forwards (ntt_forward_batch): does a 2^20 pass, whose 1024 tiles are
exactly one round of the chip's 1024 workgroup slots, lose to the lack of overlap between workgroups?

    python tools/exp_batch.py [--log-n 20] [--batches 1,2,4,8,16] [--warmup 30 --steps 50]

Prints one JSON line per batch: ms per call, ms per transform, per-launch averages (HIP events).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, action="append", default=[])
    ap.add_argument("--batches", default="1,2,4,8,16")
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    import torch
    from ntt_amd.ntt import NTTPlan
    for lg in a.log_n or [20]:
        pl = NTTPlan(1, lg, 4)
        for b in [int(x) for x in a.batches.split(",")]:
            t = pl.empty(b)
            tv = t.view(b, pl.n, -1)
            for i in range(b):
                pl.fill(tv[i], "random", seed=2 + i)
            for _ in range(a.warmup):
                pl.forward_batch(t, b)
            torch.cuda.synchronize()
            pl.set_profiling(True)
            t0 = time.perf_counter()
            for _ in range(a.steps):
                pl.forward_batch(t, b)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps * 1e3
            launches = pl.last_launch_ms()
            pl.set_profiling(False)
            print(json.dumps({"log_n": lg, "batch": b, "ms_per_call": dt, "ms_per_transform": dt / b,
                              "launch_ms": launches, "elem_per_s": b * (1 << lg) / (dt * 1e-3)}), flush=True)
            del t
        pl.close()


if __name__ == "__main__":
    main()
