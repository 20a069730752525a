"""Per-launch HIP-event timings of one plan's transform (ntt_plan_set_profiling), several configs.

    python tools/exp_launches.py [--cfg f0_L1_n26] [--cfg f1_L4_n20] ... [--warmup 50 --steps 100]

cfg = f<field>_L<limbs64>_n<log_n>[_inv][_ip][_sl][_b<k>] (ip: NTT_PLAN_IN_PLACE, sl: NTT_PLAN_SINGLE_LAUNCH,
b<k>: a batch of 2^k transforms per call, ntt_forward_batch / ntt_inverse_batch).  Prints one JSON line per cfg:
mean ms per transform (host clock around `steps` calls) and the per-launch averages, plus the
algorithmic-byte rate of each launch (one read + one write of the vector: the caller's width for
the first read / last write, the plan scratch width in between is NOT assumed -- bytes are given per
launch as 2 n S_caller for reference only).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", action="append", default=[])
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch
    from ntt_amd.ntt import NTTPlan
    rows = []
    for cfg in a.cfg or ["f0_L1_n26", "f1_L4_n20", "f1_L4_n24"]:
        m = re.fullmatch(r"f(\d)_L(\d)_n(\d+)((?:_inv|_ip|_sl)*)(?:_b(\d+))?", cfg)
        if not m:
            raise SystemExit(f"bad cfg {cfg}")
        f, L, lg, extra = int(m[1]), int(m[2]), int(m[3]), m[4]
        inv, ip, sl = "_inv" in extra, "_ip" in extra, "_sl" in extra
        bk = int(m[5]) if m[5] else 0
        pl = NTTPlan(f, lg, L, in_place=ip, single_launch=sl)
        if bk:  # the whole batch filled through a plan of its total length
            t = pl.empty(1 << bk)
            fp = NTTPlan(f, lg + bk, L)
            fp.fill(t, "random", seed=2)
            del fp
            nb = 1 << bk
            step = (lambda: pl.inverse_batch(t, nb)) if inv else (lambda: pl.forward_batch(t, nb))
        else:
            t = pl.fill(pl.empty(), "random", seed=2)
            step = (lambda: pl.inverse(t)) if inv else (lambda: pl.forward(t))
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        pl.set_profiling(True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        la = pl.last_launch_ms()
        pl.set_profiling(False)
        r = {"cfg": cfg, "ms": dt * 1e3, "elements_per_s": (1 << (lg + bk)) / dt, "passes": pl.passes, "launch_ms": la}
        rows.append(r)
        print(json.dumps(r), flush=True)
        del pl, t
        torch.cuda.empty_cache()
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
