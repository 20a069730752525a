"""Time every BASELINE.json config that fits ONE MI355X (the headline is bench.py's job).

    python tools/bench_configs.py [--out gpurun_out/configs.jsonl]

One JSON line per config:
  C2  2^20 forward, BN254 Fr (single-kernel-class size: 7+7+6 passes)
  C3  2^24 forward + inverse, BLS12-381 Fr, 4- and 6-limb element layouts
  C4  2^28 forward, BN254 Fr: on one GPU as a plain transform, and as the partitioned four-step
      with 8 virtual ranks on one device (device copies stand in for the RCCL all-to-all; the
      all-to-all over xGMI is timed only by bench.py --four-step on a multi-GPU node)
  C5  polynomial multiply of length 2^24 (2 forward + pointwise + inverse), BN254 Fr, on one GPU
      and as the distributed schedule over 8 virtual ranks
  +   2^24 coset forward (low-degree extension), BN254 Fr
Timing: W warmups, then K runs bracketed by torch.cuda.synchronize(); inputs resident in HBM.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, warmup=30, steps=20):
    # warmup covers the GPU clock ramp (~20-30 transforms at 2^24, profiles/r01_v11/ramp.txt)
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
    ap.add_argument("--out", default="gpurun_out/configs.jsonl")
    args = ap.parse_args()
    import torch
    from ntt_amd.ntt import NTTPlan
    from ntt_amd.distributed import VirtualRanks

    rows = []

    def emit(name, n, secs, **extra):
        r = {"config": name, "n": n, "ms": secs * 1e3, "elements_per_s": n / secs, **extra}
        rows.append(r)
        print(json.dumps(r), flush=True)

    # the reference's own field and entry point: SSIP over P = 469762049, long long elements
    for lg in (24, 26):
        pl = NTTPlan(0, lg, 1)
        t = pl.fill(pl.empty(), "random", seed=1)
        emit(f"SSIP path: 2^{lg} forward P469762049 (reference field, 8-B elements)", 1 << lg,
             timeit(lambda: pl.forward(t)), passes=pl.passes)
        del pl, t

    # C2
    pl = NTTPlan(1, 20, 4)
    t = pl.fill(pl.empty(), "random", seed=2)
    emit("C2: 2^20 forward BN254 Fr", 1 << 20, timeit(lambda: pl.forward(t), steps=50), passes=pl.passes)
    del pl, t
    # C2 as the reference's single-kernel class (NTT_PLAN_SINGLE_LAUNCH: one persistent launch)
    pl = NTTPlan(1, 20, 4, single_launch=True)
    t = pl.fill(pl.empty(), "random", seed=2)
    emit("C2: 2^20 forward BN254 Fr as ONE kernel (NTT_PLAN_SINGLE_LAUNCH)", 1 << 20,
         timeit(lambda: pl.forward(t), steps=50), passes=pl.passes,
         note="round 5: the two passes of 4096-element tiles with one grid barrier, a plain launch (k_fused2b); "
              "bit-exact with the default line above (DESIGN.md §4)")
    assert pl.device_status() == 0
    del pl, t
    # ... in place: BASELINE C2's "single-kernel self-sort-in-place" (no scratch, k_fused2bi)
    pl = NTTPlan(1, 20, 4, single_launch=True, in_place=True)
    t = pl.fill(pl.empty(), "random", seed=2)
    emit("C2: 2^20 forward BN254 Fr as ONE kernel in place (NTT_PLAN_SINGLE_LAUNCH | NTT_PLAN_IN_PLACE)", 1 << 20,
         timeit(lambda: pl.forward(t), steps=50), passes=pl.passes)
    assert pl.device_status() == 0
    del pl, t
    # a 3-pass single launch (grid barriers, plain launch since round 5): 2^22
    for sl in (False, True):
        pl = NTTPlan(1, 22, 4, single_launch=sl)
        t = pl.fill(pl.empty(), "random", seed=2)
        emit(f"2^22 forward BN254 Fr{' as ONE kernel (k_fused3b)' if sl else ''}", 1 << 22,
             timeit(lambda: pl.forward(t), steps=50), passes=pl.passes)
        assert pl.device_status() == 0
        del pl, t

    # C3
    for L in (4, 6):
        pl = NTTPlan(2, 24, L)
        t = pl.fill(pl.empty(), "random", seed=3)
        emit(f"C3: 2^24 forward BLS12-381 Fr, {L}x64-bit limbs", 1 << 24, timeit(lambda: pl.forward(t)), passes=pl.passes)
        emit(f"C3: 2^24 inverse BLS12-381 Fr, {L}x64-bit limbs", 1 << 24, timeit(lambda: pl.inverse(t)), passes=pl.passes)
        emit(f"C3: 2^24 forward+inverse BLS12-381 Fr, {L}x64-bit limbs", 1 << 24,
             timeit(lambda: (pl.forward(t), pl.inverse(t))), passes=pl.passes,
             note="elements_per_s counts n per forward+inverse pair")
        del pl, t
        torch.cuda.empty_cache()

    # C4
    pl = NTTPlan(1, 28, 4)
    t = pl.fill(pl.empty(), "random", seed=4)
    emit("C4: 2^28 forward BN254 Fr, one GPU (plain transform)", 1 << 28, timeit(lambda: pl.forward(t), 3, 5),
         passes=pl.passes)
    del pl, t
    torch.cuda.empty_cache()
    # NTT_PLAN_IN_PLACE (no plan scratch): palindromic passes + the tile-swap digit reversal
    for lg, (w, s) in ((24, (30, 20)), (28, (3, 5))):
        pl = NTTPlan(1, lg, 4, in_place=True)
        t = pl.fill(pl.empty(), "random", seed=4)
        emit(f"in place: 2^{lg} forward BN254 Fr (NTT_PLAN_IN_PLACE, no scratch)", 1 << lg,
             timeit(lambda: pl.forward(t), w, s), passes=pl.passes)
        del pl, t
        torch.cuda.empty_cache()
    for pieces, cpieces in ((1, 1), (4, 1), (4, 4)):
        vr = VirtualRanks(1, 28, 4, 8, pieces=pieces, col_pieces=cpieces)
        xs = vr.fill(vr.empty(), "random", seed=4)
        emit(f"C4: 2^28 forward BN254 Fr, four-step over 8 virtual ranks on one GPU, {pieces} x {cpieces} "
             f"exchange piece(s)", 1 << 28, timeit(lambda: vr.forward(xs), 2, 3), pieces=pieces, col_pieces=cpieces,
             note="exchange = device copies on one GPU (side stream, overlapping the row transforms before it "
                  "and the column transforms after it when pieces > 1); the RCCL all-to-all is timed by "
                  "bench.py --four-step")
        del vr, xs
        torch.cuda.empty_cache()

    # C5 and coset
    pl = NTTPlan(1, 24, 4)
    a = pl.fill(pl.empty(), "random", seed=5)
    b = pl.fill(pl.empty(), "random", seed=6)
    c = pl.empty()
    emit("2^24 inverse BN254 Fr", 1 << 24, timeit(lambda: pl.inverse(a)), passes=pl.passes)
    # end-to-end window: host (pinned) -> HBM, forward, HBM -> host
    h_in = a.cpu().pin_memory()
    h_out = torch.empty_like(h_in).pin_memory()

    def e2e():
        c.copy_(h_in, non_blocking=True)
        pl.forward(c)
        h_out.copy_(c, non_blocking=True)
    emit("2^24 forward BN254 Fr, end to end incl. H2D + D2H of 512 MiB each (pinned)", 1 << 24,
         timeit(e2e, 5, 10))
    del h_in, h_out
    emit("C5: polymul length 2^24 BN254 Fr (2 forward + pointwise + inverse), one GPU", 1 << 24,
         timeit(lambda: pl.polymul(a, b, c)))
    emit("coset forward 2^24 BN254 Fr (shift = generator 5)", 1 << 24, timeit(lambda: pl.forward_coset(a, 5)))
    del pl, a, b, c
    torch.cuda.empty_cache()
    for pieces in (1, 4):
        vr = VirtualRanks(1, 24, 4, 8, pieces=pieces, col_pieces=pieces)
        As = vr.fill(vr.empty(), "random", seed=5)
        Bs = vr.fill(vr.empty(), "random", seed=6)
        Cs = vr.empty()
        emit(f"C5: polymul length 2^24 BN254 Fr, distributed schedule over 8 virtual ranks on one GPU, "
             f"{pieces} x {pieces} exchange piece(s)", 1 << 24, timeit(lambda: vr.polymul(As, Bs, Cs), 5, 10),
             pieces=pieces,
             note="2 exchanges (a and b batched in one) as device copies; RCCL timing needs a multi-GPU node")
        del vr, As, Bs, Cs
        torch.cuda.empty_cache()

    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
