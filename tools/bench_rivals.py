"""Default four-step DIF schedule vs the rival schedules (the reference's bellperson / improved_NTT
family as Stockham autosort passes, NTT_PLAN_STOCKHAM; GZKP(B, G) as bit reversal + in-place DIT
passes, NTT_PLAN_GZKP; `naive` as bit reversal + one radix-2 round per launch, NTT_PLAN_NAIVE;
`naive_no_swap`, NTT_PLAN_NO_SWAP; the same bealto family kernel for kernel, NTT_PLAN_BELLPERSON and
NTT_PLAN_IMPROVED_V1..V4, one launch per round of 2^deg-point groups): forward transforms, inputs in HBM.
Per round of the bealto family: its time and the HBM rate of one read + one write of the vector.

    python tools/bench_rivals.py [--out gpurun_out/rivals.jsonl]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


BEALTO = ("bellperson", "v1", "v2", "v3", "v4")


def timeit(fn, warmup=40, steps=40):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/rivals.jsonl")
    args = ap.parse_args()
    import torch
    from ntt_amd.ntt import NTTPlan
    rows = []
    for fid, L, lg in ((1, 4, 24), (1, 4, 20), (0, 1, 24), (0, 1, 26)):
        for sched in ("default", "stockham", "gzkp", "naive", "no_swap") + BEALTO:
            pl = NTTPlan(fid, lg, L, stockham=(sched == "stockham"), gzkp=(sched == "gzkp"), naive=(sched == "naive"),
                         no_swap=(sched == "no_swap"), bealto=sched if sched in BEALTO else "")
            t = pl.fill(pl.empty(), "random", seed=1)
            pl.set_profiling(True)
            s = timeit(lambda: pl.forward(t))
            launches = pl.last_launch_ms()
            labels = pl.last_launch_labels()
            pl.set_profiling(False)
            r = {"field": fid, "limbs64": L, "log_n": lg, "schedule": sched, "passes": pl.passes, "ms": s * 1e3,
                 "elements_per_s": (1 << lg) / s, "launch_ms": launches}
            if sched == "naive" and len(launches) == 2:  # [bit reversal, the log2 n rounds]
                S = 8 * L
                r["round_ms"] = launches[1] / lg
                r["round_hbm_gbs"] = 2 * (1 << lg) * S / (r["round_ms"] * 1e-3) / 1e9  # one read + one write
            if sched in BEALTO:
                S = 8 * L
                r["labels"] = labels
                r["round_hbm_gbs"] = [round(2 * (1 << lg) * S / (ms * 1e-3) / 1e9, 1)
                                      for ms, lab in zip(launches, r["labels"]) if lab != "cp"]
            rows.append(r)
            print(json.dumps(r), flush=True)
            del pl, t
            torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
