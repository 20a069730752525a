#!/usr/bin/env python3
"""Benchmark: field-elements/sec of a 2^24-point forward NTT over BN254 Fr (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]

A "step" is one forward transform of a whole 2^24-element vector (SURVEY §8d synthetic vector B,
SplitMix64 limbs), resident in HBM when the timed region starts.

* N = 1: one MI355X, one 2^24 transform per step.
* N > 1, one rank per GPU: by default ONE 2^24 transform split over the N ranks as the four-step
  with the RCCL all-to-all ("scaling": "strong"; `value` = 2^24 / t, t = max over
  ranks).  ``--independent`` instead runs one 2^24 transform per rank with no data-path collective
  ("weak", `value` = N 2^24 / t): a secondary line, linear by construction.
  Launch: under ``torch.distributed.run`` (WORLD_SIZE set) every process is one rank.  A plain
  ``python bench.py --gpus N`` spawns the N ranks itself (torch.distributed.run in a child process,
  before any GPU call), passes rank 0's line through and exits with the children's status; it
  refuses N above the visible device count (except the one-GPU rehearsal, NTT_BENCH_EXCHANGE=host).
  The line carries `rccl_ranks` (world size of the RCCL group), `exchange_ms` /
  `exchange_gbps_per_link` (bytes each rank sends one peer per exchange / the all-to-all window) and
  `parity`: after the timed region, the transform's output gathered to rank 0 is compared element by
  element with a one-GPU plan there, plus the closed-form KAT of x_j = j at sampled k.
* ``--four-step`` at N = 1 times the partitioned schedule on one GPU (RCCL world size 1);
  ``--log-n 28 --four-step`` on 8 GPUs is BASELINE config 4.

Rank 0 prints one JSON line with
* `roofline`: SURVEY §8(d)'s transform-level HBM roofline — algorithmic bytes 2·n·S per forward
  (one read + one write of the vector) ÷ time per transform ÷ (G × 8 TB/s); `traffic` = the
  rocprofv3 PMC HBM bytes of one transform (FETCH_SIZE ×2 + WRITE_SIZE, MI355X_MICROARCH.md
  gfx950 correction) when the committed summary was measured on these kernel sources, else null.
  `roofline.dominant_kernel` = the same for the longest launch alone (HIP events on its stream
  inside the timed region);
* `valu_roofline`: that launch against the v_mad_u64_u32 issue peak (the kernels are bound by
  256-bit multiply-adds);
* `cpu_baseline`: the C oracle on the host (a bounded sample; see cpu_baseline()).
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
    """v_mad_u64_u32 issued per element in one pass of radix 2^log_r (ntt_kernels_impl.hpp, 256-bit
    class: 4 elements per thread, 4 waves per workgroup): radix-4/2 register sub-stages with 1/4, 0
    internal products per element, (Q-1)/Q twiddle products between sub-stages (Shoup) -- except in
    the wave-uniform sub-stages (sigma_s = 2^logsig(s) <= 4 waves), whose cp = 0 waves (1/sigma_s of
    them) skip theirs -- and in column passes one outer-twiddle Montgomery product.
    (Quotient-estimate reductions, 9 MADs each, are not counted.)"""
    subs, r = [], log_r
    while r > 0:
        subs.append(min(2, r))
        r -= min(2, r)
    internal = {3: 5 / 8, 2: 1 / 4, 1: 0.0}
    shoup = sum(internal[q] for q in subs)
    for s, q in enumerate(subs[:-1]):
        sig = 2 ** (log_r - 2 * s - q)  # sigma_s
        skip = 1 / sig if (s >= 1 and 2 <= sig <= 4) else 0.0
        shoup += (2 ** q - 1) / 2 ** q * (1 - skip)
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
                    help="one transform split over all ranks (four-step + RCCL all-to-all); default for N > 1")
    ap.add_argument("--pieces", default=None,
                    help="four-step: row pieces whose all-to-all overlaps the next piece's row transforms "
                         "(default 1: one whole-block exchange; 'auto': DistNTT.auto_pieces, >= 2^22 "
                         "elements per piece)")
    ap.add_argument("--col-pieces", default=None,
                    help="four-step: column pieces whose transforms start as their part of the all-to-all "
                         "arrives (default 1; 'auto')")
    ap.add_argument("--prewarm-s", type=float, default=0.3,
                    help="after --warmup, keep stepping (untimed) until the warmup lasted this long (clock ramp)")
    ap.add_argument("--no-parity", action="store_true", help="skip the post-timing parity check")
    ap.add_argument("--no-secondary", action="store_true",
                    help="N > 1: skip the secondary timings after the headline (pipelined pieces, independent "
                         "transforms per rank)")
    ap.add_argument("--independent", action="store_true",
                    help="N > 1: one independent transform per rank (weak scaling, no data-path collective)")
    ap.add_argument("--cpu-log-n", type=int, default=22, help="C-oracle single-core sample size (log2)")
    return ap.parse_args()


def _cpu_share():
    """Threads the C oracle may use: the harness's per-GPU CPU share (OMP_NUM_THREADS, 16 on the GPU
    boxes, whose os.cpu_count() counts the whole 256-thread machine) or the affinity mask."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or avail, avail


def _cpu_model() -> str:
    """The host CPU's model name (/proc/cpuinfo, SURVEY §8d: record the lscpu model)."""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.lower().startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_baseline(field_id: int, limbs: int, log_n: int):
    """The C oracle (oracle/ntt_oracle.c, a restatement of GZKP-NTT.cu:30-48) on the host: the full
    2^24 workload split over the box's CPU share (OpenMP, the multiprocess leg of SURVEY §8d), plus a
    bounded 1-core sample of the scalar restatement and the reference's own CPU NTT on its own field."""
    from oracle import oracle_c as OC
    from oracle import ntt_ref as R
    p, g = R.FIELDS[field_id]
    x = OC.random_limbs(field_id, 1 << log_n, seed=2, L=limbs)
    t0 = time.perf_counter()
    OC.ntt_mp(x, p, g)
    dt1 = time.perf_counter() - t0
    del x
    threads, avail = _cpu_share()
    big = 24
    xb = OC.random_limbs(field_id, 1 << big, seed=2, L=limbs)
    t0 = time.perf_counter()
    OC.ntt_mp_par(xb, p, g, threads)
    dtp = time.perf_counter() - t0
    cpu = _cpu_model()
    # SURVEY §8(d)'s per-config CPU runs: C1 and 2^20 in full, 2^24 once (above), 2^28 extrapolated
    # from the 2^24 run by n log n and labelled so (the reference's own CPU timings for comparison:
    # self-sort-in-place.cu:450-471, GZKP-NTT.cu:1592-1599)
    from ntt_amd import plumbing
    t0 = time.perf_counter()
    plumbing.cpu_ntt_c1(12)
    dc1 = time.perf_counter() - t0
    x = OC.random_limbs(field_id, 1 << 12, seed=1, L=limbs)
    t0 = time.perf_counter()
    OC.ntt_mp(x, p, g)
    dc1c = time.perf_counter() - t0
    x = OC.random_limbs(field_id, 1 << 20, seed=2, L=limbs)
    t0 = time.perf_counter()
    OC.ntt_mp_par(x, p, g, threads)
    d20p = time.perf_counter() - t0
    t0 = time.perf_counter()
    OC.ntt_mp(x, p, g)
    d20 = time.perf_counter() - t0
    del x
    t28 = dtp * (1 << (28 - big)) * 28 / big
    configs = {
        "C1_2^12_python": {"value": 4096 / dc1, "seconds": dc1, "cores": 1, "kind": "port",
                           "sample": "C1: 2^12-point forward NTT of x_j = j over BN254 Fr by the repo's Python CPU "
                                     "path (ntt_amd/plumbing.cpu_ntt_c1: radix-2 DIF + bit reversal), in full"},
        "C1_2^12_c": {"value": 4096 / dc1c, "seconds": dc1c, "cores": 1, "kind": "port",
                      "sample": f"2^12-point forward NTT ({FIELD_NAMES[field_id]}, SplitMix64 seed 1), scalar C "
                                "oracle, in full"},
        "2^20": {"value": (1 << 20) / d20p, "seconds": d20p, "cores": threads, "kind": "port",
                 "single_core": {"value": (1 << 20) / d20, "seconds": d20, "cores": 1},
                 "sample": f"2^20-point forward NTT ({FIELD_NAMES[field_id]}, seed 2), C oracle over {threads} "
                           "OpenMP threads and on 1 core, in full"},
        "2^24": {"value": (1 << big) / dtp, "seconds": dtp, "cores": threads, "kind": "port",
                 "sample": "the headline cpu_baseline run above, once"},
        "2^28_extrapolated": {"value": (1 << 28) / t28, "seconds": t28, "cores": threads, "kind": "port",
                              "extrapolated": True,
                              "sample": "EXTRAPOLATED, not run: the 2^24 run's time x 16 x 28/24 (n log2 n)"},
    }
    return {"value": (1 << big) / dtp, "unit": "field-elements/s", "cores": threads, "kind": "port",
            "configs": configs,
            "cpu_model": cpu,
            "sample": f"one 2^{big}-point forward NTT ({FIELD_NAMES[field_id]}, {limbs}x64-bit limbs, SplitMix64 "
                      f"input) by the C oracle split over {threads} OpenMP threads ({cpu}): {dtp:.2f} s",
            "cores_note": f"{threads} threads = this process's CPU share (OMP_NUM_THREADS / affinity {avail}); "
                          f"os.cpu_count()={os.cpu_count()} counts the whole host, which one GPU's job may not use",
            "seconds": dtp,
            "single_core": {"value": (1 << log_n) / dt1, "cores": 1, "seconds": dt1,
                            "sample": f"one 2^{log_n}-point forward NTT, scalar C oracle, 1 core"},
            "reference_field_single_core": _cpu_reference_field()}


def _cpu_reference_field(log_n: int = 22):
    """The reference's CPU path on its own field, P = 469762049, x_j = j (its input), 1 core, as the
    restatement oracle_ntt_u64 of GZKP-NTT.cu:30-48 (kind "port").  The reference's own compiled code
    (oracle/_ref) is a test-only checker and is never loaded into the bench process; the tests pin
    the port against it (tests/test_oracle_ref.py, tests/golden/ref_p469762049.npz)."""
    import numpy as np
    from oracle import oracle_c as OC
    x = np.arange(1 << log_n, dtype=np.int64)
    t0 = time.perf_counter()
    OC.ntt_u64(x, 469762049, 3)
    dt = time.perf_counter() - t0
    return {"value": (1 << log_n) / dt, "unit": "field-elements/s", "cores": 1, "seconds": dt, "kind": "port",
            "sample": f"one 2^{log_n}-point forward NTT over P469762049 (GZKP-NTT.cu:30-48 restated)"}


def load_traffic(tag: str):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary (tools/pmc_to_traffic.py) for
    this workload, only if it was measured on the current kernel sources; else (None, reason)."""
    from ntt_amd.build import source_hash
    path = os.path.join(HERE, "profiles", "pmc_summary.json")
    try:
        ent = json.load(open(path)).get(tag)
    except Exception:
        return None, "no profiles/pmc_summary.json"
    if not isinstance(ent, dict):
        return None, f"no PMC summary for {tag}"
    if ent.get("src_hash") != source_hash():
        return None, f"stale: PMC summary measured on sources {ent.get('src_hash')}, current {source_hash()}"
    return ent, ent.get("profile")


def pair_traffic(ent, labels, launch_ms):
    """PMC bytes per launch of this run, paired by launch LABEL: the summary's
    launches (tools/pmc_to_traffic.py: labels from the rocprofv3 kernel names) must be this run's
    launches (ntt_plan_last_launch_labels), same labels in the same order, one timing per launch;
    otherwise (None, reason) and no traffic is reported."""
    if not isinstance(ent, dict):
        return None, ent
    lb, ll = ent.get("launch_bytes"), ent.get("launch_labels")
    if not lb or ll is None:
        return None, "PMC entry without per-launch labels"
    if list(ll) != list(labels):
        return None, f"PMC launches {list(ll)} are not this run's launches {list(labels)}"
    if len(lb) != len(ll) or (launch_ms is not None and len(launch_ms) != len(ll)):
        return None, f"{len(lb)} PMC launches, {len(ll)} labels, {len(launch_ms or [])} timed launches"
    return list(lb), None


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def visible_devices() -> int:
    """Devices the HIP runtime would show, counted in a CHILD process, so that the launcher parent
    (spawn_ranks) never loads torch or the HIP runtime at all (the guarantee "no GPU call
    before the launcher" must not rest on what device_count() happens to do on one image)."""
    import subprocess
    code = "import torch; print(torch.cuda.device_count())"
    try:
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    except subprocess.TimeoutExpired:
        raise SystemExit("bench.py: the device-count probe (a child importing torch) did not finish in 600 s")
    try:
        if r.returncode != 0:
            raise ValueError
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        # the probe failed (not "0 devices"): say so, with the child's own error
        raise SystemExit(f"bench.py: the device-count probe failed (exit {r.returncode}):\n{r.stderr[-2000:]}")


def spawn_ranks(args) -> int:
    """``python bench.py --gpus N`` with no launcher: start the N ranks as children through
    torch.distributed.run (one process per GPU) and return their exit status.  This process makes no
    GPU call and does not import torch (visible_devices counts in a child).  rank 0's JSON line reaches
    our stdout through the inherited file descriptor."""
    import subprocess
    rehearsal = os.environ.get("NTT_BENCH_EXCHANGE", "") == "host"
    visible = visible_devices()
    if args.gpus > visible and not rehearsal:
        print(f"bench.py: --gpus {args.gpus} but only {visible} visible device(s); refusing to run "
              f"{args.gpus} ranks on fewer GPUs (NTT_BENCH_EXCHANGE=host rehearses them on one GPU)",
              file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "16"))
    return subprocess.run(cmd, env=env).returncode


def _kat_check(field_id: int, log_n: int, limbs: int, values, ks) -> bool:
    """Closed-form KAT of x_j = j (any field; the reference's own input, GZKP-NTT.cu:1587):
    X_0 = n (n - 1) / 2 and X_k = n / (w^k - 1) for k != 0, at the sampled k."""
    from ntt_amd.fields import field_params
    p, g = field_params(field_id)
    n = 1 << log_n
    w = pow(g, (p - 1) // n, p)
    for k, v in zip(ks, values):
        want = (n * (n - 1) // 2) % p if k == 0 else n * pow((pow(w, k, p) - 1) % p, p - 2, p) % p
        if v != want:
            return False
    return True


def _to_ints(rows):
    """[k, limbs] int64 host rows (or [k] for one limb) -> Python ints."""
    import numpy as np
    a = rows.cpu().numpy()
    if a.ndim == 1:
        return [int(v) for v in a]
    u = a.view(np.uint64)
    return [sum(int(u[i, j]) << (64 * j) for j in range(u.shape[1])) for i in range(u.shape[0])]


def _sample_ks(n: int):
    import random
    rng = random.Random(1234)
    return sorted({0, 1, 2, n // 2, n - 1} | {rng.randrange(n) for _ in range(59)})


def assemble_columns(parts, n1: int, c: int):
    """Column-layout shares -> the natural-order vector: rank g holds [n1][c] with element (k1, kc) =
    X[g c + kc + n2 k1] (n2 = G c), so [G][n1][c] transposed to [n1][G][c] is X in order."""
    import torch
    st = torch.stack(parts)
    tail = tuple(st.shape[2:])
    st = st.reshape((len(parts), n1, c) + tail).transpose(0, 1).contiguous()
    return st.reshape((n1 * len(parts) * c,) + tail)


def parity_four_step(args, eng, dist, rehearsal, local):
    """After the timed region: forward of SURVEY §8d vector B (seed 2) through the distributed
    schedule, gathered to rank 0 and compared with a one-GPU plan there (all n outputs), plus the
    KAT of x_j = j at sampled k.  Returns the parity dict on rank 0 (None elsewhere)."""
    import torch
    from ntt_amd.ntt import NTTPlan
    L = eng.layout
    world, rank = L.world, L.rank

    def gather_cols(t):
        if rehearsal:  # gloo: CPU tensors
            parts = [torch.empty_like(t, device="cpu") for _ in range(world)]
            dist.all_gather(parts, t.cpu())
            parts = [q.to(t.device) for q in parts]
        else:
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t)
        return assemble_columns(parts, L.n1, L.c)

    out = {}
    x = eng.empty()
    eng.fill(x, "random", seed=2)
    eng.forward(x)
    got = gather_cols(x)
    xi = eng.empty()
    eng.fill(xi, "iota", seed=0)
    eng.forward(xi)
    got_iota = gather_cols(xi)
    torch.cuda.synchronize()
    if rank == 0:
        ref = NTTPlan(field_id=args.field, log_n=args.log_n, limbs64=args.limbs, device=local)
        y = ref.empty()
        ref.fill(y, "random", seed=2)
        ref.forward(y)
        torch.cuda.synchronize()
        full_ok = torch.equal(got, y)
        ks = _sample_ks(L.n)
        idx = torch.tensor(ks, dtype=torch.int64, device=got_iota.device)
        kat_ok = _kat_check(args.field, args.log_n, args.limbs, _to_ints(got_iota[idx]), ks)
        out = {"status": "ok" if (full_ok and kat_ok) else "MISMATCH",
               "full_vs_one_gpu_plan": full_ok, "kat_iota_sampled": kat_ok,
               "checked": f"all 2^{args.log_n} forward outputs of vector B (seed 2), gathered from {world} "
                          f"rank(s) to rank 0, against a one-GPU plan on rank 0; x_j = j against the "
                          f"closed-form KAT at {len(ks)} sampled k"}
        del ref, y
    del got, got_iota, x, xi
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    return out if rank == 0 else None


def parity_single(args, plan):
    """After the timed region (N = 1 / independent ranks): x_j = j through the same plan, against the
    closed-form KAT at sampled k, and forward + inverse of vector B returning the input."""
    import torch
    if args.inverse:
        return {"status": "skipped", "reason": "parity is checked on the forward transform"}
    x = plan.empty()
    plan.fill(x, "iota", seed=0)
    plan.forward(x)
    ks = _sample_ks(plan.n)
    idx = torch.tensor(ks, dtype=torch.int64, device=x.device)
    kat_ok = _kat_check(args.field, args.log_n, args.limbs, _to_ints(x[idx]), ks)
    y = plan.empty()
    plan.fill(y, "random", seed=2)
    y0 = y.clone()
    plan.forward(y)
    plan.inverse(y)
    torch.cuda.synchronize()
    rt_ok = torch.equal(y, y0)
    return {"status": "ok" if (kat_ok and rt_ok) else "MISMATCH", "kat_iota_sampled": kat_ok,
            "round_trip_vector_b": rt_ok,
            "checked": f"x_j = j against the closed-form KAT at {len(ks)} sampled k; inverse(forward(B)) == B"}


def _timed(step, steps: int, warmup: int, barrier, dist, dev: str) -> float:
    """ms per step over `steps` calls after `warmup`, barrier + synchronize on both sides, max over ranks."""
    import torch
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    tt = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item()) / steps * 1e3


def secondary_timings(args, eng, dist, rccl, local, barrier):
    """After the headline: (a) the same distributed transform with the pipelined exchange pieces of
    DistNTT.auto_pieces, (b) one independent 2^log_n transform per rank.  Both timed like the
    headline (fewer steps), each rank's time maxed over ranks."""
    import torch
    from ntt_amd.distributed import DistNTT
    from ntt_amd.ntt import NTTPlan
    dev = f"cuda:{local}" if rccl else "cpu"
    steps, warm = max(5, min(args.steps, 30)), max(3, min(args.warmup, 20))
    n = 1 << args.log_n
    res = {}
    L = eng.layout
    ar = DistNTT.auto_pieces(L.local_n)
    ac = DistNTT.auto_pieces(L.local_n, cap=4, min_elems=DistNTT.MIN_COL_PIECE_ELEMS)
    if getattr(args, "_tuned", False):
        res["pipelined_pieces"] = {"skipped": "timed by the exchange-schedule measurement (exchange_schedule)"}
    elif (ar, ac) != (len(eng.fs.pieces), eng.fs.cp):
        e2 = DistNTT(field_id=args.field, log_n=args.log_n, limbs64=args.limbs, device=local,
                     host_exchange=not rccl, pieces="auto", col_pieces="auto")
        d2 = e2.empty()
        e2.fill(d2, "random", seed=2)
        ms = _timed(lambda: e2.forward(d2), steps, warm, barrier, dist, dev)
        res["pipelined_pieces"] = {"row_pieces": len(e2.fs.pieces), "col_pieces": e2.fs.cp, "ms_per_step": ms,
                                   "value": n / (ms * 1e-3), "steps": steps, "warmup": warm}
        del e2, d2
    else:
        res["pipelined_pieces"] = {"skipped": f"auto pieces for {L.local_n} local elements are 1 x 1"}
    pl = NTTPlan(field_id=args.field, log_n=args.log_n, limbs64=args.limbs, device=local)
    x = pl.empty()
    pl.fill(x, "random", seed=2 + L.rank)
    ms = _timed(lambda: pl.forward(x), steps, warm, barrier, dist, dev)
    res["independent"] = {"what": f"one 2^{args.log_n} transform per rank, {L.world} ranks at once (weak scaling)",
                          "ms_per_step": ms, "value": L.world * n / (ms * 1e-3), "steps": steps, "warmup": warm}
    del pl, x
    torch.cuda.synchronize()
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.independent and args.four_step:
        raise SystemExit("--independent and --four-step are exclusive")
    four_step = args.four_step or (world > 1 and not args.independent)
    # NTT_BENCH_EXCHANGE=host: rehearsal of N ranks on ONE GPU (RCCL refuses duplicate devices): the
    # all-to-all is staged through host memory over gloo.  Not a measurement of the product path.
    rehearsal = os.environ.get("NTT_BENCH_EXCHANGE", "") == "host"
    ndev = max(1, torch.cuda.device_count())
    if world > ndev and not rehearsal:
        raise SystemExit(f"{world} ranks but {ndev} visible device(s): one rank per GPU")
    # one rank per GPU; the modulo only matters when rehearsing several ranks on one device
    local = local % ndev
    torch.cuda.set_device(local)
    n = 1 << args.log_n

    use_dist = world > 1 or four_step
    rccl = False
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if four_step and not rehearsal:  # the data path exchanges over RCCL (all-to-all)
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
            rccl = True
        else:  # independent transforms (or the rehearsal): barrier / max / host exchange over gloo
            dist.init_process_group("gloo")
    if four_step:
        from ntt_amd.distributed import DistNTT
        eng = DistNTT(field_id=args.field, log_n=args.log_n, limbs64=args.limbs, device=local,
                      host_exchange=rehearsal, pieces=args.pieces, col_pieces=args.col_pieces)
        data = eng.empty()
        tuned = None
        if world > 1 and args.pieces is None and args.col_pieces is None:
            # the exchange schedule is chosen by measurement on this node (DistNTT.tune_pieces) on a
            # canonical vector, then the data is filled again
            eng.fill(data, "random", seed=2)
            tuned = eng.tune_pieces(data)
        eng.fill(data, "random", seed=2)
        step = (lambda: eng.inverse(data)) if args.inverse else (lambda: eng.forward(data))
        plan_for_prof = eng
    else:
        tuned = None
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
    # Clock ramp: the GPU's clocks settle over the first ~25 transforms, or ~0.3 s, after
    # start-up or idle; a short --warmup (the driver's 5) would time the ramp, not the steady state.
    # Keep stepping, untimed, until the warmup has lasted PREWARM_S of GPU time (reported as
    # warmup_run); the timed region below is still exactly --steps steps.
    # N > 1: the ranks decide together, chunk by chunk, so every rank runs the same steps (they exchange).
    extra, t_w = 0, time.perf_counter()
    while args.prewarm_s > 0 and extra < 4000:
        go = time.perf_counter() - t_w < args.prewarm_s
        if use_dist:
            g = torch.tensor([1 if go else 0], dtype=torch.int64, device=f"cuda:{local}" if rccl else "cpu")
            dist.all_reduce(g, op=dist.ReduceOp.MAX)
            go = bool(g.item())
        if not go:
            break
        for _ in range(8):
            step()
        extra += 8
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
    launch_labels = plan_for_prof.last_launch_labels()  # which kernel each of those launches was
    plan_for_prof.set_profiling(False)
    exchange_ms = eng.exchange_ms() if four_step else None  # mean all-to-all window per step

    elapsed = t1 - t0
    if use_dist:
        dev = f"cuda:{local}" if rccl else "cpu"
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / args.steps * 1e3
    jobs = 1 if four_step else world  # independent 2^log_n transforms per step
    value = jobs * n / (elapsed / args.steps)

    elem_bytes = 8 if args.limbs == 1 else 8 * args.limbs
    passes = list(getattr(plan_for_prof, "passes", []))
    what = "inverse" if args.inverse else "forward"
    out = {
        "metric": METRIC if (args.field == 1 and args.log_n == 24 and not args.inverse) else
        f"field-elements/sec, 2^{args.log_n} {what} NTT over {FIELD_NAMES[args.field]}",
        "value": value,
        "unit": "field-elements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_run": args.warmup + extra,  # untimed steps actually run (the clock-ramp pre-warm included)
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if four_step else "weak",
        "vs_baseline": None,
        "dtype": ("u256 mod p: 9 x 29-bit limbs, u32 x u32 + u64 MAD (v_mad_u64_u32)" if args.limbs == 4 else
                  ("u384 mod p: 14 x 29-bit limbs, u32 x u32 + u64 MAD" if args.limbs == 6 else
                   "u32 mod p (Montgomery)")),
        "data": "synthetic: SplitMix64 field elements (SURVEY §8d vector B, seed 2), resident in HBM",
        # the plan's default schedule ping-pongs through an n-element plan scratch (the caller's buffer
        # holds input and output); NTT_PLAN_IN_PLACE is the scratch-free contract of the reference's
        # SSIP (GZKP-NTT.cu:1452-1558), timed in tools/bench_configs.py
        "config": {"workload": f"2^{args.log_n}-point {what} NTT, "
                               f"{FIELD_NAMES[args.field]}, {args.limbs}x64-bit limbs, natural order, result in "
                               f"the caller's buffer (passes ping-pong through an n-element plan scratch)",
                   "log_n": args.log_n, "field": FIELD_NAMES[args.field], "limbs64": args.limbs,
                   "passes_log_radix": passes,
                   "parallelism": ((f"REHEARSAL: four-step over {world} ranks on {ndev} GPU(s), host-staged "
                                    f"gloo exchange" if rehearsal else
                                    f"four-step over {world} GPU(s) (RCCL all-to-all, one transform)") if four_step
                                   else ("single GPU" if world == 1 else
                                         f"{world} GPUs, one independent transform per rank (no data-path "
                                         f"collective)")),
                   "transforms_per_step": jobs,
                   **({"exchange_pieces": len(eng.fs.pieces), "exchange_col_pieces": eng.fs.cp,
                       "split_log_n1_n2": [eng.layout.log_n1, eng.layout.log_n2]} if four_step else {})},
        # world size of the RCCL (nccl-backend) process group carrying the data path; 0 = none
        "rccl_ranks": world if rccl else 0,
    }
    if four_step and tuned is not None:
        out["exchange_schedule"] = {**tuned, "how": "measured before the warmup: each candidate's forward "
                                    "timed on every rank (max over ranks), the fastest kept for the timed steps"}
    if four_step:
        # rank 0's all-to-all window per transform (HIP events on the compute stream around the
        # exchange: from the first piece's start to the last piece's arrival; with the default single
        # whole-block exchange it is the all-to-all alone).  Each rank sends every peer one block of
        # r c elements per exchange over that pair's link, so the per-link rate is block / window.
        out["exchange_ms"] = exchange_ms
        peer_bytes = eng.layout.chunk * elem_bytes
        out["exchange_bytes_per_peer"] = peer_bytes
        out["exchange_gbps_per_link"] = (peer_bytes / (exchange_ms * 1e-3) / 1e9
                                         if exchange_ms and world > 1 else None)
        # the convention, comparable with DESIGN §6's 77 / 153 GB/s per direction: ONE direction of one
        # peer pair's link -- the block a rank sends one peer per exchange over the window; the same
        # amount flows the other way at the same time
        out["exchange_gbps_convention"] = ("per direction: exchange_bytes_per_peer (sent to ONE peer) / exchange_ms; "
                                           "the peer sends as much back over the same link concurrently")
        if rehearsal:
            out["exchange_note"] = "host-staged gloo exchange on one GPU: not an xGMI link rate"
    # ---- SURVEY §8(d) roofline of the whole transform: 2 n S algorithmic bytes per transform
    gpus_per_transform = world if four_step else 1
    alg_transform = 2 * n * elem_bytes
    t_transform = ms_per_step * 1e-3  # every rank runs its transform(s) per step
    achieved = alg_transform / t_transform / gpus_per_transform / 1e9
    # PMC entries: one GPU's transform (tag ..._w1), or one RANK's local launches of the four-step over
    # G ranks (tag ..._w<G>_fs: rank 0 of a G-rank plan on one GPU, rows + columns, tools/pmc_ranklocal.sh;
    # kernels only -- the all-to-all's own HBM reads and writes are not in it)
    tag = (f"f{args.field}_L{args.limbs}_n{args.log_n}_w{gpus_per_transform}{'_fs' if four_step else ''}"
           f"{'_inv' if args.inverse else ''}")
    ent, prof_src = load_traffic(tag)
    launch_bytes, unpaired = pair_traffic(ent, launch_labels, launch_avg)
    if launch_bytes is None and isinstance(ent, dict):
        prof_src = f"{prof_src}: not attached, {unpaired}"
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": (sum(launch_bytes) if launch_bytes else None),
            "traffic_source": prof_src,
            "algorithmic_bytes": alg_transform / gpus_per_transform,
            "definition": "SURVEY §8(d): 2·n·S bytes per transform (one read + one write of the vector) "
                          "÷ time per transform ÷ (G × 8 TB/s); traffic = PMC HBM bytes per transform per GPU"}
    if launch_avg:
        # dominant kernel = the longest launch; algorithmic bytes per launch = one read + one write of
        # the vector it sweeps (the local share in four-step mode)
        k = max(range(len(launch_avg)), key=lambda i: launch_avg[i])
        local_n = n // world if four_step else n
        alg_bytes = 2 * local_n * elem_bytes
        ach_k = alg_bytes / (launch_avg[k] * 1e-3) / 1e9
        roof["dominant_kernel"] = {"kernel": f"launch {k} of {len(launch_avg)}" +
                                             (f" ({launch_labels[k]})" if k < len(launch_labels) else ""),
                                   "kernel_ms": launch_avg[k],
                                   "achieved": ach_k, "frac": ach_k / HBM_PEAK_GBPS,
                                   "algorithmic_bytes_per_launch": alg_bytes,
                                   "traffic": (launch_bytes[k] if launch_bytes and k < len(launch_bytes) else None)}
        roof["launch_ms"] = launch_avg
        roof["launch_labels"] = launch_labels
        if launch_bytes and len(launch_bytes) == len(launch_avg):
            out["hbm_pmc_gbps_per_gpu"] = sum(launch_bytes) / (sum(launch_avg) * 1e-3) / 1e9
        if args.limbs == 4 and args.field in (1, 2) and not four_step and len(passes) == len(launch_avg) \
                and len(passes) >= 2:
            # compute roofline of the same launch: MADs issued per launch / its duration vs the
            # v_mad_u64_u32 issue peak (the binding resource)
            mads = local_n * pass_mads(passes[k], column=k + 1 < len(passes))
            ach = mads / (launch_avg[k] * 1e-3) / 1e12
            out["valu_roofline"] = {"bound": "valu (v_mad_u64_u32 issue)", "achieved": ach, "peak": MAD_PEAK_T,
                                    "unit": "T lane-MAD/s", "frac": ach / MAD_PEAK_T,
                                    "mads_per_launch": mads, "kernel": f"launch {k} of {len(launch_avg)}"}
    out["roofline"] = roof
    # ---- parity, outside the timed region
    if not args.no_parity:
        if four_step:
            par = parity_four_step(args, eng, dist, rehearsal, local)
        else:
            par = parity_single(args, plan) if rank == 0 else None
        if rank == 0:
            out["parity"] = par
    # ---- secondary views for N > 1, outside the headline's timed region (same process group): the
    # pipelined exchange pieces (opt-in until they measurably win) and one independent transform per
    # rank (weak scaling, no data-path collective)
    if four_step and world > 1 and not args.no_secondary:
        args._tuned = tuned is not None
        sec = secondary_timings(args, eng, dist, rccl, local, barrier)
        if rank == 0:
            out["secondary"] = sec
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args.field, args.limbs if args.limbs != 1 else 1, args.cpu_log_n)
        except Exception as e:  # pragma: no cover
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.destroy_process_group()
    if rank == 0 and isinstance(out.get("parity"), dict) and out["parity"].get("status") == "MISMATCH":
        sys.exit(3)


if __name__ == "__main__":
    main()
