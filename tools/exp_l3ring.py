"""Experiment: does keeping a pass's scratch resident in the Infinity Cache (256 MiB L3) pay?

Passes 2 and 3 of the 2^24 transform are 256 independent 2^16 transforms over 2 MiB blocks.  Here
the same work runs as batched 2^16 transforms (column pass + final pass, as in the 2^24 plan):
  * one launch pair over all 256 blocks (the plan's scratch is 512 MiB: HBM round trip), vs
  * G launch pairs over 256/G blocks each (the scratch is 512/G MiB and re-used: L3-resident).
The 2^24 transform is timed beside it on the same box.

    python tools/exp_l3ring.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from ntt_amd.ntt import NTTPlan

    def timed(fn, reps=60, warm=40):
        for _ in range(warm):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    big = NTTPlan(1, 24, 4)
    t24 = big.fill(big.empty(), "random", seed=2)
    print(f"2^24 forward: {timed(lambda: big.forward(t24)):.4f} ms", flush=True)
    big.close()

    pl16 = NTTPlan(1, 16, 4)
    n = 1 << 16
    buf = t24  # 2^24 random elements = 256 blocks of 2^16
    for groups in (1, 2, 4, 8, 16, 32):
        nb = 256 // groups
        views = [buf[g * nb * n:(g + 1) * nb * n] for g in range(groups)]

        def run():
            for v in views:
                pl16.forward_batch(v, nb)
        print(f"2^16 x 256 as {groups:2d} launch pairs of {nb:3d} (scratch {nb * 2} MiB): "
              f"{timed(run):.4f} ms", flush=True)
    print(f"2^24 forward again: ", flush=True)
    pl16.close()
    big = NTTPlan(1, 24, 4)
    print(f"2^24 forward: {timed(lambda: big.forward(t24)):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
