#!/usr/bin/env python3
"""Benchmark: field-elements/sec of a 2^24-point forward NTT over BN254 Fr (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]

A "step" is one forward transform of a whole 2^24-element vector (SURVEY §8d synthetic vector B,
SplitMix64 limbs), resident in HBM when the timed region starts.

* N = 1: one MI355X, one 2^24 transform per step.
* N > 1 (torch.distributed.run, one rank per GPU): a 2^24 transform fits one GPU, and the
  north star partitions the transform only from 2^26 up.  So every rank transforms its own 2^24
  polynomial (different seeds), there is no data-path collective, and `value` = N * 2^24 / t with
  t = max over ranks ("scaling": "weak").
* --four-step: ONE transform of 2^log_n split over the N ranks with the RCCL all-to-all
  (SURVEY §8e, strong scaling; e.g. BASELINE config 4: --four-step --log-n 28 on 8 GPUs).

Rank 0 prints one JSON line with `roofline` (HBM roofline of the dominant kernel, measured with
HIP events on its launch stream inside the timed region), `valu_roofline` (the same launch against
the v_mad_u64_u32 issue peak: the kernels are bound by 256-bit multiply-adds, not by HBM; see
DESIGN.md §7) and `cpu_baseline` (the C oracle on the host, a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "field-elements/sec, 2^24 forward NTT over BN254 Fr; achieved HBM GB/s vs peak"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# v_mad_u64_u32 issue peak, 8 independent chains per wave, every SIMD busy (tools/mb_isa.hip,
# profiles/r01_mb_isa.txt): 33.8e12 lane-MADs/s
MAD_PEAK_T = 33.8
SHOUP_MADS, MONT_MADS = 143, 162  # v_mad_u64_u32 per 256-bit product (field29.hpp)


def pass_mads(log_r: int, column: bool) -> float:
    """v_mad_u64_u32 per element in one pass of radix 2^log_r (ntt_kernels_impl.hpp, 256-bit class:
    4 elements per thread): radix-4/2 register sub-stages with 1/4, 0 internal products per element,
    (Q-1)/Q twiddle products between sub-stages (Shoup), and in column passes one outer-twiddle
    Montgomery product.  (Quotient-estimate reductions, 9 MADs each, are not counted.)"""
    subs, r = [], log_r
    while r > 0:
        subs.append(min(2, r))
        r -= min(2, r)
    internal = {3: 5 / 8, 2: 1 / 4, 1: 0.0}
    shoup = sum(internal[q] for q in subs) + sum((2 ** q - 1) / 2 ** q for q in subs[:-1])
    return shoup * SHOUP_MADS + (MONT_MADS if column else 0)
FIELD_NAMES = {0: "P469762049", 1: "BN254_FR", 2: "BLS12_381_FR"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    # the first ~20-30 transforms after start-up (or after >= 0.1 s idle) run 5-20 % slower while the
    # GPU's clocks ramp (tools/exp_ramp.py, profiles/r01_v11/ramp.txt): the default warmup covers it
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--log-n", type=int, default=24)
    ap.add_argument("--field", type=int, default=1)
    ap.add_argument("--limbs", type=int, default=4)
    ap.add_argument("--inverse", action="store_true", help="time the inverse instead of the forward")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--four-step", "--dist", dest="four_step", action="store_true",
                    help="one transform split over all ranks (four-step + RCCL all-to-all)")
    ap.add_argument("--cpu-log-n", type=int, default=22, help="C-oracle sample size (log2)")
    return ap.parse_args()


def cpu_baseline(field_id: int, limbs: int, log_n: int):
    """The C oracle (oracle/ntt_oracle.c, a restatement of GZKP-NTT.cu:30-48) on the host: the full
    2^24 workload split over the box's CPU share (OpenMP, OMP_NUM_THREADS or <= 16 threads, the
    multiprocess leg of SURVEY §8d), plus a bounded 1-core sample of the scalar restatement."""
    from oracle import oracle_c as OC
    from oracle import ntt_ref as R
    p, g = R.FIELDS[field_id]
    x = OC.random_limbs(field_id, 1 << log_n, seed=2, L=limbs)
    t0 = time.perf_counter()
    OC.ntt_mp(x, p, g)
    dt1 = time.perf_counter() - t0
    del x
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, avail)
    big = 24
    xb = OC.random_limbs(field_id, 1 << big, seed=2, L=limbs)
    t0 = time.perf_counter()
    OC.ntt_mp_par(xb, p, g, threads)
    dtp = time.perf_counter() - t0
    cpu = platform.processor() or platform.machine()
    return {"value": (1 << big) / dtp, "unit": "field-elements/s", "cores": threads, "kind": "port",
            "sample": f"one 2^{big}-point forward NTT ({FIELD_NAMES[field_id]}, {limbs}x64-bit limbs, SplitMix64 "
                      f"input) by the C oracle split over {threads} OpenMP threads ({cpu}, "
                      f"os.cpu_count()={os.cpu_count()}, affinity {avail}): {dtp:.2f} s",
            "seconds": dtp,
            "single_core": {"value": (1 << log_n) / dt1, "cores": 1, "seconds": dt1,
                            "sample": f"one 2^{log_n}-point forward NTT, scalar C oracle, 1 core"},
            "reference_field_single_core": _cpu_reference_field()}


def _cpu_reference_field(log_n: int = 22):
    """The reference's own CPU path on its own field: GZKP-NTT.cu:30-48 (DIT + bit reversal over
    P = 469762049, 64-bit arithmetic) as restated by oracle_ntt_u64, 1 core, x_j = j (its input)."""
    import numpy as np
    from oracle import oracle_c as OC
    x = np.arange(1 << log_n, dtype=np.int64)
    t0 = time.perf_counter()
    OC.ntt_u64(x, 469762049, 3)
    dt = time.perf_counter() - t0
    return {"value": (1 << log_n) / dt, "unit": "field-elements/s", "cores": 1, "seconds": dt,
            "sample": f"one 2^{log_n}-point forward NTT over P469762049 (the reference's CPU NTT, restated)"}


def load_traffic(tag: str):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary for this workload (or None)."""
    path = os.path.join(HERE, "profiles", "pmc_summary.json")
    try:
        d = json.load(open(path))
        return d.get(tag)
    except Exception:
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # one rank per GPU; the modulo only matters when rehearsing several ranks on one device
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    n = 1 << args.log_n

    use_dist = world > 1 or args.four_step
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if args.four_step:  # the data path exchanges over RCCL (all-to-all)
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:  # independent transforms: the only collectives are the timing barrier and max
            dist.init_process_group("gloo")
    if args.four_step:
        from ntt_amd.distributed import DistNTT
        eng = DistNTT(field_id=args.field, log_n=args.log_n, limbs64=args.limbs, device=local)
        data = eng.empty()
        eng.fill(data, "random", seed=2)
        step = (lambda: eng.inverse(data)) if args.inverse else (lambda: eng.forward(data))
        plan_for_prof = eng
    else:
        from ntt_amd.ntt import NTTPlan
        plan = NTTPlan(field_id=args.field, log_n=args.log_n, limbs64=args.limbs, device=local)
        data = plan.empty()
        plan.fill(data, "random", seed=2 + rank)  # each rank its own polynomial
        step = (lambda: plan.inverse(data)) if args.inverse else (lambda: plan.forward(data))
        plan_for_prof = plan

    def barrier():
        if use_dist:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # ---- timed region: K steps bracketed by barrier + synchronize; per-launch HIP events recorded
    # on the launch stream between kernels (ntt_plan_set_profiling) accumulate per-launch times.
    plan_for_prof.set_profiling(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    launch_avg = plan_for_prof.last_launch_ms()  # per-launch average over the timed steps (<= 64)
    plan_for_prof.set_profiling(False)

    elapsed = t1 - t0
    if use_dist:
        dev = f"cuda:{local}" if args.four_step else "cpu"
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / args.steps * 1e3
    jobs = 1 if args.four_step else world  # independent 2^log_n transforms per step
    value = jobs * n / (elapsed / args.steps)

    elem_bytes = 8 if args.limbs == 1 else 8 * args.limbs
    passes = list(getattr(plan_for_prof, "passes", []))
    out = {
        "metric": METRIC if (args.field == 1 and args.log_n == 24 and not args.inverse) else
        f"field-elements/sec, 2^{args.log_n} {'inverse' if args.inverse else 'forward'} NTT over "
        f"{FIELD_NAMES[args.field]}",
        "value": value,
        "unit": "field-elements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.four_step else "weak",
        "vs_baseline": None,
        "dtype": ("u256 mod p: 9 x 29-bit limbs, u32 x u32 + u64 MAD (v_mad_u64_u32)" if args.limbs == 4 else
                  ("u384 mod p: 14 x 29-bit limbs, u32 x u32 + u64 MAD" if args.limbs == 6 else
                   "u32 mod p (Montgomery)")),
        "data": "synthetic: SplitMix64 field elements (SURVEY §8d vector B, seed 2), resident in HBM",
        "config": {"workload": f"2^{args.log_n}-point {'inverse' if args.inverse else 'forward'} NTT, "
                               f"{FIELD_NAMES[args.field]}, {args.limbs}x64-bit limbs, natural order, in place",
                   "log_n": args.log_n, "field": FIELD_NAMES[args.field], "limbs64": args.limbs,
                   "passes_log_radix": passes,
                   "parallelism": (f"four-step over {world} GPU(s) (RCCL all-to-all)" if args.four_step else
                                   ("single GPU" if world == 1 else
                                    f"{world} GPUs, one independent transform per rank (no data-path collective)")),
                   "transforms_per_step": jobs},
    }
    if launch_avg:
        # dominant kernel = the longest launch; algorithmic bytes per launch = one read + one write
        # of the local vector (2*n*S per pass over all n elements).
        k = max(range(len(launch_avg)), key=lambda i: launch_avg[i])
        local_n = n // world if args.four_step else n
        alg_bytes = 2 * local_n * elem_bytes
        achieved = alg_bytes / (launch_avg[k] * 1e-3) / 1e9
        tag = f"f{args.field}_L{args.limbs}_n{args.log_n}_w{world if args.four_step else 1}"
        traffic = load_traffic(tag)
        out["roofline"] = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                           "frac": achieved / HBM_PEAK_GBPS,
                           "traffic": traffic[k] if isinstance(traffic, list) and k < len(traffic) else None,
                           "kernel": f"launch {k} of {len(launch_avg)}", "kernel_ms": launch_avg[k],
                           "algorithmic_bytes_per_launch": alg_bytes,
                           "launch_ms": launch_avg}
        total_alg = 2 * local_n * elem_bytes * max(1, len(launch_avg))
        out["hbm_effective_gbps_per_gpu"] = total_alg / (ms_per_step * 1e-3) / 1e9
        if args.limbs == 4 and args.field in (1, 2) and not args.four_step and len(passes) == len(launch_avg) \
                and len(passes) >= 2:
            # compute roofline of the same launch: MADs issued per launch / its duration vs the
            # v_mad_u64_u32 issue peak (the binding resource)
            mads = local_n * pass_mads(passes[k], column=k + 1 < len(passes))
            ach = mads / (launch_avg[k] * 1e-3) / 1e12
            out["valu_roofline"] = {"bound": "valu (v_mad_u64_u32 issue)", "achieved": ach, "peak": MAD_PEAK_T,
                                    "unit": "T lane-MAD/s", "frac": ach / MAD_PEAK_T,
                                    "mads_per_launch": mads, "kernel": f"launch {k} of {len(launch_avg)}"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args.field, args.limbs if args.limbs != 1 else 1, args.cpu_log_n)
        except Exception as e:  # pragma: no cover
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
