"""The exit-time SIGSEGV of processes that made a cooperative launch under rocprofv3.

    rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 tools/exit_crash_probe.py MAPS_OUT [--coop 1|0]

Runs a few single-launch transforms (the grid-barrier form at 2^19, BN254: k_fused3b, a cooperative
launch when NTT_FUSED_COOP is 1, a plain launch when 0), then, at Python exit (before the C runtime's
exit handlers and static destructors run), writes /proc/self/maps to MAPS_OUT.  A crash trace's
absolute addresses are then resolved against that map into (library, offset) pairs, which
tools/symbolize_trace.py turns into function names with llvm-symbolizer (the GPU box runs this same
image, so the libraries are the ones in /opt/rocm here).
"""
from __future__ import annotations

import argparse
import atexit
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("maps_out")
    ap.add_argument("--coop", default="1")
    ap.add_argument("--log-n", type=int, default=19)
    a = ap.parse_args()
    os.environ["NTT_FUSED_COOP"] = a.coop  # read once, at the first single launch
    import torch
    from ntt_amd.ntt import NTTPlan

    def dump_maps():
        with open("/proc/self/maps") as src, open(a.maps_out, "w") as dst:
            dst.write(src.read())

    atexit.register(dump_maps)
    ref = NTTPlan(1, a.log_n, 4)
    one = NTTPlan(1, a.log_n, 4, single_launch=True)
    x = ref.fill(ref.empty(), "random", seed=7)
    y, z = x.clone(), x.clone()
    ref.forward(y)
    for _ in range(5):
        z.copy_(x)
        one.forward(z)
    torch.cuda.synchronize()
    ok = torch.equal(y, z)
    print(f"single launch 2^{a.log_n} (NTT_FUSED_COOP={a.coop}): {'ok' if ok else 'MISMATCH'}", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
