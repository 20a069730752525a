"""Multi-GPU NTT: four-step decomposition with one all-to-all.

n = n1 * n2 (n1 >= n2; the rank plan picks the split, Layout), j = j1 + n1*j2, k = k2 + n2*k1:

    X[k2 + n2 k1] = sum_j1 w_n1^(j1 k1) * w_n^(j1 k2) * sum_j2 w_n2^(j2 k2) x[j1 + n1 j2]

Rank g of G (one process per GPU, ``torch.distributed`` over RCCL) owns

* input, "row layout":     rows j1 in [g r, (g+1) r), r = n1/G; local [r][n2], element (a, j2) = x[g r + a + n1 j2]
* output, "column layout": cols k2 in [g c, (g+1) c), c = n2/G; local [n1][c], element (k1, kc) = X[g c + kc + n2 k1]

Forward (libntt ``ntt_rplan_*``, ntt_amd/csrc/ntt_rplan.cpp) = batched n2-point NTTs of the local rows
whose last pass multiplies by w_n^(j1 k2) and stores straight into per-peer chunks -> ONE all-to-all
(RCCL; each peer chunk r*c elements) -> c interleaved n1-point NTTs that read the chunks where they
arrived.  No separate twiddle, pack or transpose pass.  The inverse mirrors it (column layout in, row
layout out), so forward / inverse / pointwise products never leave the distributed layouts.

Polynomial multiply (BASELINE config 5): forward(a) and forward(b) pack into one send buffer
[G][2][r*c] so that ONE all-to-all carries both; the pointwise product is local and fused into the
first column pass of the inverse; the inverse's all-to-all returns c = a*b to the row layout.  Three
transforms, two exchanges.

The reference has no multi-GPU code at all (no NCCL/MPI); this is new.
The orchestration (FourStep) is engine- and transport-agnostic so the same code runs with the
HIP rank plan over RCCL on GPUs, with G "virtual ranks" in one process on one GPU (exchange =
device copies), and with a CPU test engine over gloo.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Callable, List, Optional

import torch


@dataclass
class Layout:
    """n = n1 n2 over ``world`` ranks.  ``log_n2`` None: the balanced split (n2 = 2^floor(L/2)); the
    rank plans pick their own (ntt_rplan_info: fewest passes, then the smallest largest radix, then the
    most balanced; 2^24 on the 256-bit engines: 16 + 8) and pass it here."""
    log_n: int
    world: int
    rank: int
    log_n2: Optional[int] = None

    def __post_init__(self):
        if self.world < 1 or self.world & (self.world - 1):
            raise ValueError("world size must be a power of two")
        self.log_g = self.world.bit_length() - 1
        if self.log_n2 is None:
            self.log_n2 = self.log_n // 2
        self.log_n1 = self.log_n - self.log_n2
        if self.log_n2 > self.log_n1 or self.log_n2 < 0:
            raise ValueError(f"bad split 2^{self.log_n1} x 2^{self.log_n2}")
        if self.log_g > self.log_n2:
            raise ValueError(f"2^{self.log_n} is too small to split over {self.world} ranks")
        self.log_r = self.log_n1 - self.log_g  # local rows (row layout)
        self.log_c = self.log_n2 - self.log_g  # local columns (column layout)
        self.n = 1 << self.log_n
        self.n1, self.n2 = 1 << self.log_n1, 1 << self.log_n2
        self.r, self.c = 1 << self.log_r, 1 << self.log_c
        self.local_n = self.n >> self.log_g
        self.chunk = self.r * self.c  # elements per peer chunk of one vector

    # global index of local element i (tests / fills)
    def row_global(self, i: int) -> int:
        a, j2 = i >> self.log_n2, i & (self.n2 - 1)
        return self.rank * self.r + a + self.n1 * j2

    def col_global(self, i: int) -> int:
        k1, kc = i >> self.log_c, i & (self.c - 1)
        return self.rank * self.c + kc + self.n2 * k1


def pow2_pieces(k, limit: int) -> int:
    """The piece count actually used: the largest power of two <= min(k, limit) (pieces are uniform,
    so that every exchange unit is one contiguous run of the buffer layouts below)."""
    k = max(1, min(int(k), int(limit)))
    return 1 << (k.bit_length() - 1)


class FourStep:
    """Per-rank four-step schedule over an engine (local compute) and an exchange (all-to-all).

    The local steps run in pieces so that the all-to-all overlaps compute on BOTH sides of it:
    P_r row pieces (r / P_r rows each) and P_c column pieces (c / P_c columns each, both powers of two).

    * forward: the row transforms of row piece i are exchanged while those of piece i + 1 run; the
      last row piece goes out column piece by column piece, and the column transforms of piece k start
      as soon as its part has arrived (the earlier row pieces are in by then);
    * inverse: mirrored -- the column transforms of column piece k are exchanged while piece k + 1
      transforms; the last column piece goes out row piece by row piece, and the inverse row
      transforms of piece i start as soon as its part has arrived.

    A column piece is c / P_c whole length-n1 transforms and a row piece r / P_r whole length-n2
    transforms, so no transform ever waits for more than its own inputs.  Exchange buffers hold one
    block of nvec * r * c elements per peer (ntt.h, ntt_rplan_*_piece):

    * forward blocks [i][v][k][r / P_r][c / P_c]: row piece i of every vector is one contiguous run,
      and so is each (i, v, k) unit;
    * inverse blocks [k][i][r / P_r][c / P_c] (nvec = 1): column piece k is one run, and so is each
      (k, i) unit.

    With P_r = P_c = 1 both are [G][nvec][r][c].

    Engine interface (one rank): ``forward_rows_piece(x, send, nvec, slot, i, P_r, P_c)``,
    ``forward_cols_piece(recv, x, nvec, slot, k, P_r, P_c)``, ``inverse_cols_piece(x, y, send, k,
    P_r, P_c)`` (column layout, times y if given), ``inverse_rows_piece(recv, out, i, P_r, P_c)``,
    ``empty(count)``.  Exchange interface: ``start(send, recv, peer_stride, runs)`` moves the runs
    [(offset, length), ...] (elements, relative to each peer's block of ``peer_stride`` elements) from
    every rank to every rank, ordered after the compute enqueued so far, and returns a handle;
    ``wait(handle)`` orders later compute after it.  A plain callable ``exchange(send, recv)`` (one
    all-to-all of whole blocks) is accepted too and runs the schedule unpipelined.
    """

    def __init__(self, layout: Layout, engine, exchange=None, pieces: int = 1, col_pieces: int = 1):
        self.L = layout
        self.eng = engine
        if exchange is not None and not hasattr(exchange, "start"):
            exchange, pieces, col_pieces = _WholeExchange(exchange), 1, 1
        self.exchange = exchange
        self.rp = pow2_pieces(pieces, layout.r)
        self.cp = pow2_pieces(col_pieces, layout.c)
        ra = layout.r // self.rp
        self.pieces = [(i * ra, ra) for i in range(self.rp)]  # row pieces (first row, rows)
        self.send = engine.empty(layout.local_n)
        self.recv = engine.empty(layout.local_n)
        self.send2 = self.recv2 = None  # the polymul's two-vector exchange buffers, on first use

    @staticmethod
    def piece_ranges(r: int, pieces: int):
        """Near-equal row ranges (the row-range entry points ntt_rplan_*_rows_range, ntt_mplan)."""
        k = max(1, min(int(pieces), r))
        step = -(-r // k)
        return [(a, min(step, r - a)) for a in range(0, r, step)]

    def pair_buffers(self):
        if self.send2 is None:
            self.send2 = self.eng.empty(2 * self.L.local_n)
            self.recv2 = self.eng.empty(2 * self.L.local_n)
        return self.send2, self.recv2

    # ---- exchange units (element runs within one peer block)
    def fwd_runs(self, nvec, i, k=None):
        L = self.L
        ra, cm = L.r // self.rp, L.c // self.cp
        base = i * nvec * ra * L.c
        if k is None:
            return [(base, nvec * ra * L.c)]
        return [(base + v * ra * L.c + k * ra * cm, ra * cm) for v in range(nvec)]

    def inv_runs(self, k, i=None):
        L = self.L
        ra, cm = L.r // self.rp, L.c // self.cp
        base = k * L.r * cm
        return [(base, L.r * cm)] if i is None else [(base + i * ra * cm, ra * cm)]

    # ---- forward: row layout -> column layout (in place on each x)
    def _forward(self, xs, send, recv):
        nvec, ps = len(xs), len(xs) * self.L.chunk
        early, tail = [], []
        for i in range(self.rp):
            for v, x in enumerate(xs):
                self.eng.forward_rows_piece(x, send, nvec, v, i, self.rp, self.cp)
            if i < self.rp - 1 or self.cp == 1:
                early.append(self.exchange.start(send, recv, ps, self.fwd_runs(nvec, i)))
            else:
                tail = [self.exchange.start(send, recv, ps, self.fwd_runs(nvec, i, k)) for k in range(self.cp)]
        for h in early:
            self.exchange.wait(h)
        for k in range(self.cp):
            if tail:
                self.exchange.wait(tail[k])
            for v, x in enumerate(xs):
                self.eng.forward_cols_piece(recv, x, nvec, v, k, self.rp, self.cp)

    def forward(self, x):
        self._forward([x], self.send, self.recv)
        return x

    # ---- inverse: column layout (times y) -> row layout in out
    def _inverse(self, x, y, out):
        ps = self.L.chunk
        early, tail = [], []
        for k in range(self.cp):
            self.eng.inverse_cols_piece(x, y, self.send, k, self.rp, self.cp)
            if k < self.cp - 1 or self.rp == 1:
                early.append(self.exchange.start(self.send, self.recv, ps, self.inv_runs(k)))
            else:
                tail = [self.exchange.start(self.send, self.recv, ps, self.inv_runs(k, i)) for i in range(self.rp)]
        for h in early:
            self.exchange.wait(h)
        for i in range(self.rp):
            if tail:
                self.exchange.wait(tail[i])
            self.eng.inverse_rows_piece(self.recv, out, i, self.rp, self.cp)
        return out

    def inverse(self, x):
        return self._inverse(x, None, x)

    # ---- polynomial multiply: row-layout a, b -> row-layout out = a * b (cyclic, length n).
    # a and b are left holding their column-layout forward transforms (unless out aliases them).
    def polymul(self, a, b, out):
        if a is b:  # squaring: one forward, single-vector exchange
            self.forward(a)
        else:
            send2, recv2 = self.pair_buffers()
            self._forward([a, b], send2, recv2)  # a and b in every exchange unit
        return self._inverse(a, b, out)


def tune_four_step(layout: Layout, engine, exchange, dist, group, x, candidates, steps: int, warmup: int,
                   device, sync: Callable[[], None]):
    """Time forward(x) under each candidate (row pieces, column pieces) on every rank of `group`, in
    the same order on every rank; a candidate's time is the slowest rank's (all_reduce MAX), so every
    rank picks the same schedule.  Returns (the fastest FourStep, {"chosen", "ms_per_transform", ...})."""
    import time as _t
    results, best = {}, None
    for p, q in candidates:
        fs = FourStep(layout, engine, exchange, pieces=p, col_pieces=q)
        for _ in range(warmup):
            fs.forward(x)
        sync()
        dist.barrier(group=group)
        t0 = _t.perf_counter()
        for _ in range(steps):
            fs.forward(x)
        sync()
        dt = torch.tensor([(_t.perf_counter() - t0) / max(1, steps)], dtype=torch.float64, device=device)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=group)
        key = f"{len(fs.pieces)}x{fs.cp}"
        results[key] = float(dt.item()) * 1e3
        if best is None or results[key] < best[0]:
            best = (results[key], fs, key)
    return best[1], {"chosen": best[2], "ms_per_transform": results, "steps": steps, "warmup": warmup}


class _WholeExchange:
    """Adapter for a plain ``exchange(send, recv)`` callable: whole-block all-to-all, one piece."""

    def __init__(self, fn):
        self.fn = fn

    def start(self, send, recv, peer_stride, runs):
        self.fn(send, recv)

    def wait(self, handle):
        pass


def run_views(buf, world: int, peer_stride: int, runs):
    """[peer][run] views of an exchange buffer: run (off, len) of every peer block."""
    return [[buf[g * peer_stride + off:g * peer_stride + off + ln] for off, ln in runs] for g in range(world)]


class RankPlan:
    """libntt ``ntt_rplan``: one rank's fused local steps on one GPU (the product path)."""

    def __init__(self, field_id: int, log_n: int, limbs64: int, world: int, rank: int, device: int):
        from . import lib as _L
        self._L = _L
        self.lib = _L.load()
        self.limbs64 = limbs64
        self.device = device
        h = C.c_void_p()
        _L.check(self.lib.ntt_rplan_create(C.byref(h), field_id, log_n, limbs64, world, rank, device),
                 "ntt_rplan_create")
        self.handle = h
        n1, n2 = C.c_uint(), C.c_uint()
        _L.check(self.lib.ntt_rplan_info(h, None, None, C.byref(n1), C.byref(n2), None), "ntt_rplan_info")
        self.layout = Layout(log_n, world, rank, n2.value)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            self.lib.ntt_rplan_destroy(h)
            self.handle = None

    def empty(self, count: int) -> torch.Tensor:
        shape = (count,) if self.limbs64 == 1 else (count, self.limbs64)
        return torch.empty(shape, dtype=torch.int64, device=f"cuda:{self.device}")

    @staticmethod
    def _p(t):
        return C.c_void_p(t.data_ptr()) if t is not None else None

    def _s(self, t):
        return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)

    def forward_rows(self, x, send, nvec, slot, row0=0, nrows=None):
        """Rows [row0, row0 + nrows) -> [G][nvec][r][c] blocks (the row-range entry point, ntt_mplan's layout)."""
        nrows = self.layout.r - row0 if nrows is None else nrows
        self._L.check(self.lib.ntt_rplan_forward_rows_range(self.handle, self._p(x), self._p(send), nvec, slot, row0,
                                                            nrows, self._s(x)), "ntt_rplan_forward_rows_range")

    def forward_cols(self, recv, x, nvec, slot):
        self._L.check(self.lib.ntt_rplan_forward_cols(self.handle, self._p(recv), self._p(x), nvec, slot, self._s(x)),
                      "ntt_rplan_forward_cols")

    def inverse_cols(self, x, y, send):
        self._L.check(self.lib.ntt_rplan_inverse_cols(self.handle, self._p(x), self._p(y), self._p(send), self._s(x)),
                      "ntt_rplan_inverse_cols")

    def inverse_rows(self, recv, out, row0=0, nrows=None):
        nrows = self.layout.r - row0 if nrows is None else nrows
        self._L.check(self.lib.ntt_rplan_inverse_rows_range(self.handle, self._p(recv), self._p(out), row0, nrows,
                                                            self._s(out)), "ntt_rplan_inverse_rows_range")

    # ---- the piece entry points FourStep schedules (ntt_rplan_*_piece)
    def forward_rows_piece(self, x, send, nvec, slot, i, rp, cp):
        self._L.check(self.lib.ntt_rplan_forward_rows_piece(self.handle, self._p(x), self._p(send), nvec, slot, i, rp,
                                                            cp, self._s(x)), "ntt_rplan_forward_rows_piece")

    def forward_cols_piece(self, recv, x, nvec, slot, k, rp, cp):
        self._L.check(self.lib.ntt_rplan_forward_cols_piece(self.handle, self._p(recv), self._p(x), nvec, slot, k, rp,
                                                            cp, self._s(x)), "ntt_rplan_forward_cols_piece")

    def inverse_cols_piece(self, x, y, send, k, rp, cp):
        self._L.check(self.lib.ntt_rplan_inverse_cols_piece(self.handle, self._p(x), self._p(y), self._p(send), k, rp,
                                                            cp, self._s(x)), "ntt_rplan_inverse_cols_piece")

    def inverse_rows_piece(self, recv, out, i, rp, cp):
        self._L.check(self.lib.ntt_rplan_inverse_rows_piece(self.handle, self._p(recv), self._p(out), i, rp, cp,
                                                            self._s(out)), "ntt_rplan_inverse_rows_piece")

    def fill(self, t, kind: str = "random", seed: int = 1):
        k = {"iota": 0, "random": 1}[kind]
        self._L.check(self.lib.ntt_rplan_fill(self.handle, self._p(t), k, int(seed), self._s(t)), "ntt_rplan_fill")
        return t

    def set_profiling(self, enable: bool = True) -> None:
        self._L.check(self.lib.ntt_rplan_set_profiling(self.handle, int(bool(enable))), "ntt_rplan_set_profiling")

    def last_launch_ms(self, which: int) -> List[float]:
        buf = (C.c_float * 16)()
        k = C.c_uint()
        self._L.check(self.lib.ntt_rplan_last_launch_ms(self.handle, which, buf, 16, C.byref(k)),
                      "ntt_rplan_last_launch_ms")
        return [buf[i] for i in range(k.value)]

    def last_launch_labels(self, which: int) -> List[str]:
        buf = C.create_string_buffer(256)
        self._L.check(self.lib.ntt_rplan_last_launch_labels(self.handle, which, buf, 256),
                      "ntt_rplan_last_launch_labels")
        v = buf.value.decode()
        return v.split(",") if v else []

    def profile_group(self) -> None:
        self._L.check(self.lib.ntt_rplan_profile_group(self.handle), "ntt_rplan_profile_group")


class DistNTT:
    """One rank of a distributed NTT: the fused rank plan + torch.distributed all-to-all (RCCL on GPUs).

    The default process group must be initialised (``nccl`` backend = RCCL on ROCm).  ``forward``
    takes this rank's row-layout share and leaves its column-layout share in place; ``inverse`` the
    reverse.  See module docstring for the layouts.  The all-to-all runs in units of ``pieces`` row
    pieces x ``col_pieces`` column pieces, each an asynchronous RCCL all-to-all on the communicator's
    stream, overlapping the local transforms on both sides of the exchange (FourStep).
    """

    # Default: ONE whole-block exchange per transform (1 x 1 pieces).  On one GPU the pieces never
    # measured a clear gain: 2^24 over 2 virtual ranks 2.18 / 2.16 / 2.21 ms for 1x1 / 2x1 / 4x4, and
    # C4 over 8 with 4 x 4 pieces ran 33.4 ms in one refresh and 43.4 / 45.0 ms in the next two while
    # C5 with 4 x 4 was slower than 1 x 1 (9.75 vs 8.82 ms; profiles/r03_final/configs.jsonl).  The
    # virtual-rank exchange is device copies competing with the transforms for the same HBM, so what
    # pieces hide over xGMI is only measurable on a multi-GPU node; until then they are opt-in
    # (``pieces`` / ``col_pieces``, bench.py --pieces / --col-pieces).  When enabled, a piece's row
    # transforms must still fill the GPU (one 1024-element tile per workgroup; 256 CUs x 4 resident
    # workgroups), hence the minimum piece sizes below.
    MIN_PIECE_ELEMS = 1 << 22
    MIN_COL_PIECE_ELEMS = 1 << 21

    @classmethod
    def auto_pieces(cls, local_n: int, cap: int = 8, min_elems: Optional[int] = None) -> int:
        """Largest power-of-two piece count (<= cap) keeping >= min_elems elements per piece; used only
        when pieces are requested as "auto" (DistNTT(pieces="auto"))."""
        m = cls.MIN_PIECE_ELEMS if min_elems is None else min_elems
        k = 1
        while k < cap and local_n // (2 * k) >= m:
            k *= 2
        return k

    def __init__(self, field_id: int = 1, log_n: int = 24, limbs64: int = 4, device: Optional[int] = None,
                 group=None, host_exchange: bool = False, pieces: Optional[int] = None,
                 col_pieces: Optional[int] = None):
        """host_exchange: stage the all-to-all through host memory over a gloo group (rehearsing
        several ranks on ONE GPU, where RCCL refuses duplicate devices); never the product path.
        pieces / col_pieces: row / column pieces of the pipelined exchange (None: 1, one whole-block
        exchange; "auto": auto_pieces of the local share, >= 2^22 elements per row piece, >= 2^21 per
        column piece, at most 4 of those)."""
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.host_exchange = host_exchange
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        if device is None:
            device = torch.cuda.current_device()
        self.device = device
        self.field_id, self.log_n, self.limbs64 = field_id, log_n, limbs64
        self.engine = RankPlan(field_id, log_n, limbs64, world, rank, device)
        self.layout = self.engine.layout
        ln = self.layout.local_n  # world 1: no exchange to hide
        auto_r = 1 if world == 1 else self.auto_pieces(ln)
        auto_c = 1 if world == 1 else self.auto_pieces(ln, cap=4, min_elems=self.MIN_COL_PIECE_ELEMS)
        pieces = 1 if pieces is None else (auto_r if pieces == "auto" else int(pieces))
        col_pieces = 1 if col_pieces is None else (auto_c if col_pieces == "auto" else int(col_pieces))
        self.fs = FourStep(self.layout, self.engine, self, pieces=pieces, col_pieces=col_pieces)
        self.n = self.layout.n
        self.passes: List[int] = []  # per-transform schedules: see the row / column plans
        # exchange timing (set_profiling): one window per all-to-all, from the first piece's start to
        # the last piece's arrival, as HIP events on the compute stream (so a window that overlaps
        # row transforms of later pieces includes them)
        self._x_windows: Optional[list] = None
        self._x_open: Optional[list] = None

    @classmethod
    def piece_candidates(cls, layout: Layout):
        """The exchange schedules tune_pieces measures: 1 x 1, two pieces on either side of the
        exchange and on both (2 x 1, 1 x 2, 2 x 2), and the auto_pieces size rule -- each clipped to the
        rows / columns a rank owns, duplicates dropped.  Round 4's list was 1 x 1 plus the size rule
        only, which at 2^24 over 8 ranks (2^21 elements per rank, below both piece minimums) left the
        single candidate 1 x 1: the "measured choice" measured nothing.  At world
        size 1 there is no exchange to hide: 1 x 1 only."""
        if layout.world == 1:
            return [(1, 1)]
        auto = (cls.auto_pieces(layout.local_n),
                cls.auto_pieces(layout.local_n, cap=4, min_elems=cls.MIN_COL_PIECE_ELEMS))
        out = []
        for p, q in [(1, 1), (2, 1), (1, 2), (2, 2), auto]:
            c = (pow2_pieces(p, layout.r), pow2_pieces(q, layout.c))
            if c not in out:
                out.append(c)
        return out

    def tune_pieces(self, x: torch.Tensor, candidates=None, steps: int = 8, warmup: int = 3) -> dict:
        """Plan-time measurement of the exchange schedule (FFTW_MEASURE-style; tune_four_step): every
        rank times forward(x) under each of piece_candidates(), and the fastest becomes this plan's
        schedule.  Whether pieces pay depends on the link rate against the local transforms, which only
        the node at hand can say.  Collective over the group; x is overwritten."""
        L = self.layout
        if candidates is None:
            candidates = self.piece_candidates(L)
        dev = torch.device("cpu") if self.host_exchange else x.device
        self.fs, res = tune_four_step(L, self.engine, self, self.dist, self.group, x, candidates, steps, warmup,
                                      dev, torch.cuda.synchronize)
        return res

    # RCCL moves < 2 GiB per peer per collective (a 2 GiB chunk arrived half copied,
    # tests/test_gpu_fullsize.py): larger per-peer runs go as several all-to-alls.
    MAX_PEER_BYTES = 1 << 30

    # ---- FourStep exchange interface: runs of every peer block
    def start(self, send, recv, peer_stride, runs):
        L = self.layout
        if self._x_windows is not None and (self._x_open is None or self._x_open[1] is not None):
            if self._x_open is not None:
                self._x_windows.append(self._x_open)
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            self._x_open = [e0, None]
        sv = run_views(send, L.world, peer_stride, runs)
        rv = run_views(recv, L.world, peer_stride, runs)
        works = []
        for u in range(len(runs)):
            ins = [sv[g][u] for g in range(L.world)]
            outs = [rv[g][u] for g in range(L.world)]
            if self.host_exchange:
                hr = torch.empty((L.world * ins[0].shape[0],) + tuple(ins[0].shape[1:]), dtype=ins[0].dtype)
                self.dist.all_to_all_single(hr, torch.cat(ins).cpu(), group=self.group)
                for g, o in enumerate(outs):
                    o.copy_(hr[g * o.shape[0]:(g + 1) * o.shape[0]])
                continue
            rows_b = ins[0][0:1].numel() * 8  # bytes per element
            step = max(1, self.MAX_PEER_BYTES // rows_b)
            for off in range(0, ins[0].shape[0], step):
                works.append(self.dist.all_to_all([o[off:off + step] for o in outs],
                                                  [t[off:off + step] for t in ins], group=self.group,
                                                  async_op=True))
        return works

    def wait(self, works):
        for w in works:
            w.wait()
        if self._x_windows is not None and self._x_open is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._x_open[1] = e1

    def exchange_ms(self) -> Optional[float]:
        """Mean all-to-all window (ms) over the exchanges since set_profiling(True)."""
        done = self._x_windows if self._x_windows is not None else getattr(self, "_x_frozen", [])
        wins = list(done) + ([self._x_open] if self._x_open and self._x_open[1] else [])
        if not wins:
            return None
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in wins) / len(wins)

    def empty(self) -> torch.Tensor:
        return self.engine.empty(self.layout.local_n)

    def fill(self, t: torch.Tensor, kind: str = "random", seed: int = 1) -> torch.Tensor:
        """This rank's row-layout share of the global synthetic vector (same values as NTTPlan.fill)."""
        return self.engine.fill(t, kind, seed)

    # every call is one timing group of the rank plan (ntt_rplan_profile_group): last_launch_ms then
    # reports each launch of the call, e.g. the two 2^15-row launches of the row transform at world size 1
    def forward(self, t: torch.Tensor) -> torch.Tensor:
        self.engine.profile_group()
        return self.fs.forward(t)

    def inverse(self, t: torch.Tensor) -> torch.Tensor:
        self.engine.profile_group()
        return self.fs.inverse(t)

    def polymul(self, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """Row-layout shares a, b -> row-layout share of c = a * b (cyclic, length n); two all-to-alls."""
        self.engine.profile_group()
        return self.fs.polymul(a, b, out)

    def set_profiling(self, enable: bool = True) -> None:
        """Per-launch timing of the rank plan and, from here on, exchange windows (exchange_ms);
        disabling stops recording but keeps what was measured."""
        self.engine.set_profiling(enable)
        if enable:
            self._x_windows, self._x_open = [], None
        elif self._x_windows is not None:
            if self._x_open is not None and self._x_open[1] is not None:
                self._x_windows.append(self._x_open)
            self._x_open = None
            self._x_frozen = self._x_windows
            self._x_windows = None

    def last_launch_ms(self) -> List[float]:
        """Row-transform launches, then column-transform launches (separate timing rings), of the
        latest call."""
        return self.engine.last_launch_ms(0) + self.engine.last_launch_ms(1)

    def last_launch_labels(self) -> List[str]:
        """The same launches' labels (ntt.h ntt_plan_last_launch_labels)."""
        return self.engine.last_launch_labels(0) + self.engine.last_launch_labels(1)


class _RankList:
    """G rank plans driven as one FourStep engine: every argument is a list with one tensor per rank
    (y may be None), so the schedule interleaves the G ranks step by step on the current stream."""

    def __init__(self, engines):
        self.engines = engines

    def empty(self, count):
        return [e.empty(count) for e in self.engines]

    def forward_rows_piece(self, x, send, nvec, slot, i, rp, cp):
        for e, xg, sg in zip(self.engines, x, send):
            e.forward_rows_piece(xg, sg, nvec, slot, i, rp, cp)

    def forward_cols_piece(self, recv, x, nvec, slot, k, rp, cp):
        for e, rg, xg in zip(self.engines, recv, x):
            e.forward_cols_piece(rg, xg, nvec, slot, k, rp, cp)

    def inverse_cols_piece(self, x, y, send, k, rp, cp):
        for g, e in enumerate(self.engines):
            e.inverse_cols_piece(x[g], None if y is None else y[g], send[g], k, rp, cp)

    def inverse_rows_piece(self, recv, out, i, rp, cp):
        for e, rg, og in zip(self.engines, recv, out):
            e.inverse_rows_piece(rg, og, i, rp, cp)


class VirtualRanks:
    """G ranks of the four-step in ONE process on one GPU; the all-to-all is device copies.

    SURVEY §4: validate the distributed decomposition on a single GPU before RCCL.  The schedule is
    FourStep's, over all G ranks at once; with pieces > 1 each exchange unit's copies run on a side
    stream while the next piece's transforms run.
    """

    def __init__(self, field_id: int, log_n: int, limbs64: int, world: int, device: int = 0, pieces: int = 1,
                 col_pieces: Optional[int] = None, batched: bool = False):
        """col_pieces: column pieces (None: as many as row pieces).  batched: every exchange unit's
        copies as one multi-tensor copy (torch._foreach_copy_) instead of one device copy each."""
        self.world = world
        self.batched = batched
        self.engines = [RankPlan(field_id, log_n, limbs64, world, g, device) for g in range(world)]
        self.layout0 = self.engines[0].layout
        self.layouts = [e.layout for e in self.engines]
        self.fs = FourStep(self.layout0, _RankList(self.engines), self, pieces=pieces,
                           col_pieces=pieces if col_pieces is None else col_pieces)
        self.pieces = self.fs.pieces
        self.side = torch.cuda.Stream(device=device)

    # ---- FourStep exchange interface over the G ranks' buffers (lists)
    def start(self, sends, recvs, peer_stride, runs):
        """Runs of every (src -> dst) block, on the side stream after the work enqueued so far; returns
        the event that marks their arrival."""
        G = self.world
        ev = torch.cuda.Event()
        ev.record()
        self.side.wait_event(ev)
        with torch.cuda.stream(self.side):
            sv = [run_views(t, G, peer_stride, runs) for t in sends]
            rv = [run_views(t, G, peer_stride, runs) for t in recvs]
            pairs = [(rv[dst][src][u], sv[src][dst][u]) for dst in range(G) for src in range(G)
                     for u in range(len(runs))]
            if self.batched:  # one multi-tensor copy launch instead of G*G*runs blit kernels
                torch._foreach_copy_([d for d, _ in pairs], [s for _, s in pairs])
            else:
                for d, s in pairs:
                    d.copy_(s)
            done = torch.cuda.Event()
            done.record()
        for t in list(sends) + list(recvs):  # the side stream uses them: keep the caching allocator honest
            t.record_stream(self.side)
        return done

    def wait(self, ev):
        torch.cuda.current_stream().wait_event(ev)

    def empty(self) -> List[torch.Tensor]:
        return [e.empty(self.layout0.local_n) for e in self.engines]

    def fill(self, xs: List[torch.Tensor], kind: str = "random", seed: int = 1):
        for e, t in zip(self.engines, xs):
            e.fill(t, kind, seed)
        return xs

    def forward(self, xs: List[torch.Tensor]):
        return self.fs.forward(xs)

    def inverse(self, xs: List[torch.Tensor]):
        return self.fs.inverse(xs)

    def polymul(self, As: List[torch.Tensor], Bs: List[torch.Tensor], Outs: List[torch.Tensor]):
        if all(a is b for a, b in zip(As, Bs)):
            Bs = As  # squaring: one forward, single-vector exchange
        return self.fs.polymul(As, Bs, Outs)


class MultiPlan:
    """Single-process multi-GPU plan over the C ABI (``ntt_mplan_*``, ntt_amd/csrc/ntt_multi.cpp):
    one process drives ``devices`` with the same four-step and layouts as DistNTT, the exchange
    being one grouped RCCL all-to-all.  Shares are torch tensors, ``xs[g]`` on ``devices[g]``.
    """

    def __init__(self, field_id: int = 1, log_n: int = 24, limbs64: int = 4, devices: Optional[List[int]] = None,
                 pieces: Optional[int] = None, col_pieces: Optional[int] = None):
        """pieces / col_pieces: row / column pieces of the pipelined exchange (None, None: the plan's
        default; pieces alone: row pieces only, ntt_mplan_set_pieces; both: ntt_mplan_set_pieces2)."""
        from . import lib as _L
        self._L = _L
        self.lib = _L.load()
        self.devices = list(devices if devices is not None else range(torch.cuda.device_count()))
        self.limbs64 = limbs64
        arr = (C.c_int * len(self.devices))(*self.devices)
        h = C.c_void_p()
        _L.check(self.lib.ntt_mplan_create(C.byref(h), field_id, log_n, limbs64, len(self.devices), arr),
                 "ntt_mplan_create")
        self.handle = h
        local_n, n1, n2 = C.c_uint64(), C.c_uint(), C.c_uint()
        self.lib.ntt_mplan_info(h, C.byref(local_n), C.byref(n1), C.byref(n2))
        self.local_n, self.log_n1, self.log_n2 = local_n.value, n1.value, n2.value
        self.layouts = [Layout(log_n, len(self.devices), g, self.log_n2) for g in range(len(self.devices))]
        if col_pieces is not None:
            _L.check(self.lib.ntt_mplan_set_pieces2(h, int(pieces or 1), int(col_pieces)), "ntt_mplan_set_pieces2")
        elif pieces is not None:
            _L.check(self.lib.ntt_mplan_set_pieces(h, int(pieces)), "ntt_mplan_set_pieces")

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            self.lib.ntt_mplan_destroy(h)
            self.handle = None

    def empty(self) -> List[torch.Tensor]:
        shape = (self.local_n,) if self.limbs64 == 1 else (self.local_n, self.limbs64)
        return [torch.empty(shape, dtype=torch.int64, device=f"cuda:{d}") for d in self.devices]

    def _ptrs(self, xs):
        for t, d in zip(xs, self.devices):
            if not t.is_contiguous() or t.device.index != d or t.numel() * 8 != self.local_n * 8 * self.limbs64:
                raise ValueError("each share must be a contiguous tensor of local_n elements on its device")
        data = (C.c_void_p * len(xs))(*[t.data_ptr() for t in xs])
        streams = (C.c_void_p * len(xs))(*[torch.cuda.current_stream(d).cuda_stream for d in self.devices])
        return data, streams

    def fill(self, xs, kind: str = "random", seed: int = 1):
        data, streams = self._ptrs(xs)
        self._L.check(self.lib.ntt_mplan_fill(self.handle, data, 0 if kind == "iota" else 1, seed, streams),
                      "ntt_mplan_fill")
        return xs

    def forward(self, xs):
        data, streams = self._ptrs(xs)
        self._L.check(self.lib.ntt_forward_multi(self.handle, data, streams), "ntt_forward_multi")
        return xs

    def inverse(self, xs):
        data, streams = self._ptrs(xs)
        self._L.check(self.lib.ntt_inverse_multi(self.handle, data, streams), "ntt_inverse_multi")
        return xs

    def polymul(self, As, Bs, Outs):
        """Row-layout shares of a, b -> row-layout shares of c = a * b (ntt_polymul_multi)."""
        a, streams = self._ptrs(As)
        b, _ = self._ptrs(Bs)
        c, _ = self._ptrs(Outs)
        self._L.check(self.lib.ntt_polymul_multi(self.handle, a, b, c, streams), "ntt_polymul_multi")
        return Outs
