"""Default and GZKP(B,G) schedules back to back at 2^24 BN254 (a few forwards each), for a
rocprofv3 --pmc comparison of their big-table passes (tools/pmc_rival.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from ntt_amd.ntt import NTTPlan
    for gz in (False, True):
        pl = NTTPlan(1, 24, 4, gzkp=gz)
        t = pl.fill(pl.empty(), "random", seed=2)
        for _ in range(5):
            pl.forward(t)
        torch.cuda.synchronize()
        del pl, t
    print("ok", flush=True)


if __name__ == "__main__":
    main()
