"""2^24 in two passes (12 + 12 on 4096-element tiles, NTT_TWO_PASS_24=1): bit-exact check against the
same plan's batched path (8 + 8 + 8 on 1024-element tiles), then per-launch HIP-event timings.

    NTT_TWO_PASS_24=1 python tools/exp_two_pass.py [--fid 1] [--steps 100]

Prints one JSON line: parity of forward / inverse on iota and random vectors, and the two schedules'
ms per transform (batch-1 call on the two-pass plan, a batch of two on the three-pass tiles / 2).
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
    ap.add_argument("--fid", type=int, default=1)
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--steps", type=int, default=100)
    a = ap.parse_args()
    import torch
    from ntt_amd.ntt import NTTPlan
    pl = NTTPlan(a.fid, a.log_n, 4)
    n = pl.n
    res = {"fid": a.fid, "log_n": a.log_n, "passes": pl.passes}
    b = pl.empty(2)
    bv = b.view(2, n, -1)
    ok = True
    for kind in ("iota", "random"):
        pl.fill(bv[0], kind, seed=5)
        pl.fill(bv[1], "random", seed=6)
        x0, x1 = bv[0].clone(), bv[1].clone()
        pl.set_profiling(True)
        pl.forward(x0)
        res[f"launches_{kind}"] = len(pl.last_launch_ms())
        pl.forward(x1)
        pl.set_profiling(False)
        pl.forward_batch(b, 2)
        f_ok = torch.equal(bv[0], x0) and torch.equal(bv[1], x1)
        pl.inverse(x0)
        pl.inverse(x1)
        pl.inverse_batch(b, 2)
        i_ok = torch.equal(bv[0], x0) and torch.equal(bv[1], x1)
        res[f"fwd_{kind}"] = f_ok
        res[f"inv_{kind}"] = i_ok
        ok = ok and f_ok and i_ok
    res["device_status"] = pl.device_status()
    print(json.dumps(res), flush=True)
    if not ok or res["device_status"]:
        sys.exit(1)

    t = pl.fill(pl.empty(), "random", seed=2)

    def timed(step, steps):
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        pl.set_profiling(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        la = pl.last_launch_ms()
        pl.set_profiling(False)
        return dt * 1e3, la

    for rep in range(2):
        ms1, la1 = timed(lambda: pl.forward(t), a.steps)
        ms2, la2 = timed(lambda: pl.forward_batch(b, 2), a.steps // 2)
        print(json.dumps({"rep": rep, "batch1_ms": ms1, "batch1_launch_ms": la1, "batch2_ms_per_transform": ms2 / 2,
                          "batch2_launch_ms": la2}), flush=True)


if __name__ == "__main__":
    main()
