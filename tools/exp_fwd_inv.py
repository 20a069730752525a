"""Experiment: per-call time of the 2^24 forward and inverse in different call orders and on
different input distributions (is the forward/inverse gap in configs.jsonl data, order or clock?).

    python tools/exp_fwd_inv.py [field_id]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from ntt_amd.ntt import NTTPlan

    fid = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    pl = NTTPlan(fid, 24, 4)
    t = pl.fill(pl.empty(), "random", seed=3)
    pristine = t.clone()

    def run(name, seq, reps=10, reset=False):
        ev = []
        for _ in range(2):
            for f in seq:
                f(t)
        torch.cuda.synchronize()
        ms = [[] for _ in seq]
        for _ in range(reps):
            for i, f in enumerate(seq):
                if reset:
                    t.copy_(pristine)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                f(t)
                b.record()
                ev.append((i, a, b))
        torch.cuda.synchronize()
        for i, a, b in ev:
            ms[i].append(a.elapsed_time(b))
        print(name, [f"{sorted(m)[len(m) // 2]:.3f}" for m in ms], flush=True)

    F, I = pl.forward, pl.inverse
    run("F only", [F])
    run("I only", [I])
    run("F,I pairs", [F, I])
    run("F only again", [F])
    run("F on fresh masked-random input (reset each call)", [F], reset=True)
    run("I on fresh masked-random input (reset each call)", [I], reset=True)
    # uniform [0,p) input: the forward of the masked input
    F(pristine)
    run("F on fresh uniform input (reset each call)", [F], reset=True)


if __name__ == "__main__":
    main()
