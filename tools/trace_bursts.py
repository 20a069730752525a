"""Split a rocprofv3 kernel trace of tools/bench_configs.py into the bursts of exchange copies (the
virtual-rank configs: `__amd_rocclr_copyBuffer` kernels separated by > GAP ms) and report, per burst,
its span, the NTT and copy busy time, their overlap, and the hardware queues of each.

    python tools/trace_bursts.py DIR/run_kernel_trace.csv [--gap-ms 20]"""
import csv
import sys
from collections import Counter

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_overlap import intersect, length, union  # noqa: E402


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    gap = float(sys.argv[sys.argv.index("--gap-ms") + 1]) * 1e6 if "--gap-ms" in sys.argv else 20e6
    cps = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows
                 if "copyBuffer" in r["Kernel_Name"])
    bursts, cur = [], []
    for c in cps:
        if cur and c[0] - cur[-1][1] > gap:
            bursts.append(cur)
            cur = []
        cur.append(c)
    if cur:
        bursts.append(cur)
    for i, b in enumerate(bursts):
        lo, hi = b[0][0], max(x[1] for x in b)
        ntt = [(max(int(r["Start_Timestamp"]), lo), min(int(r["End_Timestamp"]), hi)) for r in rows
               if "copyBuffer" not in r["Kernel_Name"] and int(r["End_Timestamp"]) > lo and int(r["Start_Timestamp"]) < hi]
        nq = Counter(r["Queue_Id"] for r in rows if "copyBuffer" not in r["Kernel_Name"]
                     and int(r["End_Timestamp"]) > lo and int(r["Start_Timestamp"]) < hi)
        un, uc = union(ntt), union([(x[0], x[1]) for x in b])
        print({"burst": i, "copies": len(b), "span_ms": round((hi - lo) / 1e6, 2), "ntt_busy_ms": round(length(un) / 1e6, 2),
               "copy_busy_ms": round(length(uc) / 1e6, 2), "both_ms": round(intersect(un, uc) / 1e6, 2),
               "copy_queues": dict(Counter(x[2] for x in b)), "ntt_queues": dict(nq)})


if __name__ == "__main__":
    main()
