"""Reference point for HBM-bound passes: device-to-device copy bandwidth (read + write bytes / time)
of torch's copy kernel at the NTT vector sizes.

    python tools/exp_copy_bw.py
"""
import torch


def main():
    for mib in (128, 512, 2048):
        n = mib << 20
        a = torch.empty(n, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        for _ in range(30):
            b.copy_(a)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 50
        e0.record()
        for _ in range(reps):
            b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"copy {mib} MiB: {ms:.4f} ms, {2 * n / ms / 1e6:.0f} GB/s (read + write)", flush=True)


if __name__ == "__main__":
    main()
