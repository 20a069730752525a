"""Four-step split experiment: G virtual ranks on one GPU with the rank plans' split (or the one forced
by NTT_FS_LOG_N2), checked against the one-GPU transform, then timed.

    NTT_FS_LOG_N2=8 python tools/exp_split.py [log_n] [world] [reps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from ntt_amd.distributed import VirtualRanks
    from ntt_amd.ntt import NTTPlan

    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    ref = NTTPlan(1, log_n, 4)
    x = ref.fill(ref.empty(), "random", seed=9)
    ref.forward(x)
    vr = VirtualRanks(1, log_n, 4, world)
    lay = vr.layout0
    xs = vr.fill(vr.empty(), "random", seed=9)
    vr.forward(xs)
    ok = True
    for lay, t in zip(vr.layouts, xs):
        L = lay
        i = torch.arange(L.local_n, dtype=torch.int64, device="cuda:0")
        idx = L.rank * L.c + (i & (L.c - 1)) + L.n2 * (i >> L.log_c)
        ok = ok and torch.equal(t, x[idx])
    del x, ref
    for _ in range(5):
        vr.forward(xs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        vr.forward(xs)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    rows = vr.engines[0].last_launch_ms(0)
    print(f"2^{log_n} over {world} virtual rank(s), split n1 2^{lay.log_n1} x n2 2^{lay.log_n2}: "
          f"{'OK' if ok else 'MISMATCH'} {ms:.3f} ms", flush=True)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
