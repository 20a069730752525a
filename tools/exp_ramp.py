"""Experiment: per-call forward time over the first few hundred calls after plan creation, and
after an idle second (clock ramp / power-state warm-up vs a one-time cost).

    python tools/exp_ramp.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from ntt_amd.ntt import NTTPlan

    pl = NTTPlan(1, 24, 4)
    t = pl.fill(pl.empty(), "random", seed=2)

    def curve(name, calls):
        ev = []
        for _ in range(calls):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            pl.forward(t)
            b.record()
            ev.append((a, b))
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in ev]
        chunks = [ms[i:i + 10] for i in range(0, len(ms), 10)]
        print(name, " ".join(f"{sum(c) / len(c):.3f}" for c in chunks), flush=True)

    curve("after plan creation, 10-call means:", 300)
    time.sleep(1.0)
    curve("after 1 s idle:", 100)
    time.sleep(0.1)
    curve("after 0.1 s idle:", 100)


if __name__ == "__main__":
    main()
