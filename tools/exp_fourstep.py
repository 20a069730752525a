"""Four-step breakdown at C4's size on one GPU: 2^28 BN254 forward over 8 virtual ranks (device-copy
exchange), a few timed repetitions; run under rocprofv3 --kernel-trace --stats for per-kernel times.

    python tools/exp_fourstep.py [log_n] [world] [pieces]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from ntt_amd.distributed import VirtualRanks

    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 28
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    pieces = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    vr = VirtualRanks(1, log_n, 4, world, pieces=pieces)
    xs = vr.fill(vr.empty(), "random", seed=4)
    for _ in range(2):
        vr.forward(xs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        vr.forward(xs)
    torch.cuda.synchronize()
    print(f"four-step 2^{log_n} over {world} virtual ranks, {pieces} piece(s): "
          f"{(time.perf_counter() - t0) / reps * 1e3:.2f} ms",
          flush=True)


if __name__ == "__main__":
    main()
