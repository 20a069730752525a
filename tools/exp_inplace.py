"""A/B: NTT_PLAN_IN_PLACE (no plan scratch) against the default schedule: BN254 Fr forward at 2^24
and 2^28, the SSIP field P at 2^24 and 2^26 (run under rocprofv3 --kernel-trace --stats for the per-kernel split)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, warmup, steps):
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
    import torch
    from ntt_amd.ntt import NTTPlan
    for fid, L, lg, w, s in ((1, 4, 24, 40, 40), (1, 4, 28, 3, 6), (0, 1, 24, 40, 40), (0, 1, 26, 20, 20)):
        for in_place in (False, True, False, True):
            pl = NTTPlan(fid, lg, L, in_place=in_place)
            t = pl.fill(pl.empty(), "random", seed=1)
            ms = timeit(lambda: pl.forward(t), w, s) * 1e3
            print(json.dumps({"field_id": fid, "log_n": lg, "in_place": in_place, "passes": pl.passes, "ms": ms}), flush=True)
            del pl, t
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
