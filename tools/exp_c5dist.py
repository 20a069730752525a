"""C5 over 8 virtual ranks on one GPU: is the distributed polymul host-bound or GPU-bound?

Times vr.polymul / vr.forward in a fresh process (wall time per call, host time to enqueue one call
with the GPU still busy), then cProfiles the host side of a few calls.  Usage on the box:
    python tools/exp_c5dist.py [--log-n 24] [--pieces 1] > gpurun_out/c5dist.txt
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--pieces", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batched", action="store_true", help="one multi-tensor copy per exchange unit")
    ap.add_argument("--ops", default="polymul,forward")
    ap.add_argument("--no-profile", action="store_true")
    args = ap.parse_args()
    import torch
    from ntt_amd.distributed import VirtualRanks

    vr = VirtualRanks(1, args.log_n, 4, args.world, pieces=args.pieces, col_pieces=args.pieces,
                      batched=args.batched)
    As = vr.fill(vr.empty(), "random", seed=5)
    Bs = vr.fill(vr.empty(), "random", seed=6)
    Cs = vr.empty()
    ops = {"polymul": lambda: vr.polymul(As, Bs, Cs), "forward": lambda: vr.forward(As)}
    print(f"log_n {args.log_n} world {args.world} pieces {args.pieces} x {args.pieces} batched {args.batched}")
    for name in args.ops.split(","):
        fn = ops[name]
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.steps * 1e3
        # host enqueue time of one call while the GPU is still busy with the previous ones
        hs = []
        for _ in range(args.steps):
            h0 = time.perf_counter()
            fn()
            hs.append(time.perf_counter() - h0)
        torch.cuda.synchronize()
        hs.sort()
        print(f"{name}: wall {wall:.3f} ms/call, host enqueue median {hs[len(hs) // 2] * 1e3:.3f} ms/call",
              flush=True)
    if args.no_profile:
        return
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        ops["polymul"]()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
