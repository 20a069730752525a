"""Overlap of the exchange copies with the transforms in a rocprofv3 kernel trace (VirtualRanks: the
exchange = device-to-device copies, which ROCm runs as `__amd_rocclr_copyBuffer` blit kernels).

    python tools/trace_overlap.py DIR/run_kernel_trace.csv [--last-ms 120]

Over the trace's last window (the timed transforms): per hardware queue, busy time of the NTT kernels
and of the copy kernels, the time both ran at once, and the window's wall time.  Copies and
transforms overlap only when they sit on different hardware queues."""
import csv
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    out, cur = [], None
    for a, b in iv:
        if cur and a <= cur[1]:
            cur[1] = max(cur[1], b)
        else:
            if cur:
                out.append(cur)
            cur = [a, b]
    if cur:
        out.append(cur)
    return out


def length(iv):
    return sum(b - a for a, b in iv)


def intersect(x, y):
    i = j = 0
    tot = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    path = sys.argv[1]
    last_ms = float(sys.argv[sys.argv.index("--last-ms") + 1]) if "--last-ms" in sys.argv else 120.0
    rows = list(csv.DictReader(open(path)))
    end = max(int(r["End_Timestamp"]) for r in rows)
    lo = end - int(last_ms * 1e6)
    ntt, cp = [], []
    queues = defaultdict(lambda: [0, 0])
    for r in rows:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if b < lo:
            continue
        a = max(a, lo)
        is_copy = "copyBuffer" in r["Kernel_Name"]
        (cp if is_copy else ntt).append((a, b))
        queues[r["Queue_Id"]][1 if is_copy else 0] += b - a
    un, uc = union(ntt), union(cp)
    first = min(x[0] for x in un + uc)
    print({"window_ms": (end - first) / 1e6, "ntt_busy_ms": length(un) / 1e6, "copy_busy_ms": length(uc) / 1e6,
           "both_ms": intersect(un, uc) / 1e6,
           "per_queue_ms (ntt, copy)": {q: (round(v[0] / 1e6, 2), round(v[1] / 1e6, 2)) for q, v in queues.items()}})


if __name__ == "__main__":
    main()
