"""Per-phase timing of the two-pass single launch: with NTT_FUSED_TRACE=<file>,
k_fused2b / k_fused2bi write per workgroup the 100 MHz wall clock at start, after pass 1, after the
pass barrier and at the end.  This runs `calls` single-launch forwards of 2^20 BN254 (scratch and in
place), then reports per call (median over calls after the first `skip`), relative to the earliest
start of the launch, in microseconds:
  start_spread   last workgroup start - first
  p1_end         pass 1 done: min / median / max over workgroups
  released       barrier released: min / median / max
  barrier        median release - latest pass-1 end (fan-in + poll + acquire)
  fin            end - release, median over workgroups (final pass)
  total          latest end - earliest start

    python tools/exp_fused_trace.py [--calls 50] [--out trace.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics as st
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def summarise(rec):
    nwg = rec["nwg"]
    s = rec["stamps"]
    t = [[s[4 * b + k] for k in range(4)] for b in range(nwg)]
    t0 = min(x[0] for x in t)
    us = lambda v: (v - t0) / 100.0  # 100 MHz ticks -> us
    p1 = sorted(us(x[1]) for x in t)
    rel = sorted(us(x[2]) for x in t)
    fin = sorted((x[3] - x[2]) / 100.0 for x in t)
    return {
        "start_spread": us(max(x[0] for x in t)),
        "p1_end_min": p1[0], "p1_end_med": st.median(p1), "p1_end_max": p1[-1],
        "released_min": rel[0], "released_med": st.median(rel), "released_max": rel[-1],
        "barrier": st.median(rel) - p1[-1],
        "fin_med": st.median(fin),
        "total": us(max(x[3] for x in t)),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--skip", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    path = a.out or os.path.join(tempfile.mkdtemp(), "trace.jsonl")
    if os.path.exists(path):
        os.remove(path)
    os.environ["NTT_FUSED_TRACE"] = path  # read at the first single launch
    import torch
    from ntt_amd.ntt import NTTPlan
    res = {}
    for ip in (False, True):
        pl = NTTPlan(1, 20, 4, single_launch=True, in_place=ip)
        x = pl.fill(pl.empty(), "random", seed=5)
        for _ in range(a.calls):
            pl.forward(x)
        torch.cuda.synchronize()
        del pl
    recs = [json.loads(l) for l in open(path)]
    for kern in ("k_fused2b", "k_fused2bi"):
        rs = [summarise(r) for r in recs if r["kernel"] == kern][a.skip:]
        if not rs:
            continue
        res[kern] = {k: round(st.median(r[k] for r in rs), 2) for k in rs[0]}
        res[kern]["calls"] = len(rs)
        print(json.dumps({"kernel": kern, **res[kern]}), flush=True)


if __name__ == "__main__":
    main()
