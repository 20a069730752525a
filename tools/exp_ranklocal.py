"""Rank-local work of the distributed four-step on ONE GPU: rank 0 of a
G-rank plan (ntt_rplan, world = G) for 2^log_n, timing the forward's row launches and column
launches with no exchange (the send buffer is fed to the column transforms as if it had arrived),
against 1/G of the plain one-GPU transform measured in the same process.

    python tools/exp_ranklocal.py [--log-n 24] [--worlds 1,2,4,8] [--steps 100] [--out F]

One JSON line per world: host ms per (rows + cols) over `steps` calls, the HIP-event launch
averages (rows, cols), the split, and the ratio to plain / G.
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
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--field", type=int, default=1)
    ap.add_argument("--limbs", type=int, default=4)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--inverse", action="store_true")
    ap.add_argument("--no-plain", action="store_true", help="skip the one-GPU plan (PMC runs: rank-local launches only)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch
    from ntt_amd.ntt import NTTPlan
    from ntt_amd.distributed import RankPlan

    def timed(step, n):
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    rows = []
    plain = float("nan")
    if not a.no_plain:
        pl = NTTPlan(a.field, a.log_n, a.limbs)
        t = pl.fill(pl.empty(), "random", seed=2)
        plain = timed(lambda: pl.forward(t), a.steps)
        rec = {"what": "plain", "log_n": a.log_n, "ms": plain}
        print(json.dumps(rec), flush=True)
        rows.append(rec)
        del pl, t
        torch.cuda.empty_cache()
    for G in [int(w) for w in a.worlds.split(",")]:
        rp = RankPlan(a.field, a.log_n, a.limbs, G, 0, 0)
        L = rp.layout
        x = rp.fill(rp.empty(L.local_n), "random", seed=3)
        send = rp.empty(L.local_n)
        if a.inverse:
            def step():
                rp.inverse_cols(x, None, send)
                rp.inverse_rows(send, x)
        else:
            def step():
                rp.forward_rows(x, send, 1, 0)
                rp.forward_cols(send, x, 1, 0)
        ms = timed(step, a.steps)
        rp.set_profiling(True)
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        lr, lc = rp.last_launch_ms(0), rp.last_launch_ms(1)
        rp.set_profiling(False)
        rec = {"what": "rank_local", "world": G, "log_n": a.log_n, "inverse": a.inverse,
               "log_n1": L.log_n1, "log_n2": L.log_n2, "local_n": L.local_n, "ms": ms,
               "rows_launch_ms": lr, "cols_launch_ms": lc, "launch_sum_ms": sum(lr) + sum(lc),
               "plain_over_g_ms": plain / G, "ratio": ms / (plain / G)}
        print(json.dumps(rec), flush=True)
        rows.append(rec)
        del rp, x, send
        torch.cuda.empty_cache()
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
