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
    rank plans pick their own (ntt_rplan_info: balanced unless a narrower n2 takes fewer passes) and
    pass it here."""
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


class FourStep:
    """Per-rank four-step schedule over an engine (local compute) and an exchange (all-to-all).

    Engine interface (one rank): ``forward_rows(x, send, nvec, slot, row0, nrows)`` (rows [row0,
    row0 + nrows) of the row layout -> their runs of every peer chunk), ``forward_cols(recv, x, nvec,
    slot)`` (received chunks -> column layout), ``inverse_cols(x, y, send)`` (column layout, times y
    if given -> peer chunks), ``inverse_rows(recv, out, row0, nrows)`` (-> rows of the row layout),
    ``empty(count)``.  Buffers hold [G][nvec][r][c] elements (a peer chunk is [r][c]).

    Exchange interface: ``start(send, recv, nvec, row0, nrows)`` moves rows [row0, row0 + nrows) of
    every peer chunk (all nvec vectors) and returns a handle, ordered after the compute enqueued so
    far; ``wait(handle)`` orders later compute after it.  A plain callable ``exchange(send, recv)``
    (one all-to-all of whole chunks) is accepted too and runs the schedule unpipelined.

    With ``pieces`` > 1 the row steps run in pieces of r / pieces rows: the forward exchanges each
    piece while the row transforms of the next one run, the inverse transforms each piece as soon as
    it has arrived -- the all-to-all overlaps the local transforms instead of following them.
    """

    def __init__(self, layout: Layout, engine, exchange=None, pieces: int = 1):
        self.L = layout
        self.eng = engine
        if exchange is not None and not hasattr(exchange, "start"):
            exchange, pieces = _WholeExchange(exchange), 1
        self.exchange = exchange
        self.pieces = self.piece_ranges(layout.r, pieces)
        self.send = engine.empty(layout.local_n)
        self.recv = engine.empty(layout.local_n)
        self.send2 = self.recv2 = None  # [G][2][chunk]: the polymul's batched exchange, on first use

    @staticmethod
    def piece_ranges(r: int, pieces: int):
        k = max(1, min(int(pieces), r))
        step = -(-r // k)
        return [(a, min(step, r - a)) for a in range(0, r, step)]

    def pair_buffers(self):
        if self.send2 is None:
            self.send2 = self.eng.empty(2 * self.L.local_n)
            self.recv2 = self.eng.empty(2 * self.L.local_n)
        return self.send2, self.recv2

    # ---- forward: row layout -> column layout (in place on x)
    def forward_rows_piece(self, x, i, nvec=1, slot=0, send=None):
        a0, ra = self.pieces[i]
        self.eng.forward_rows(x, self.send if send is None else send, nvec, slot, a0, ra)

    def forward(self, x):
        hs = []
        for i, (a0, ra) in enumerate(self.pieces):
            self.forward_rows_piece(x, i)
            hs.append(self.exchange.start(self.send, self.recv, 1, a0, ra))
        for h in hs:
            self.exchange.wait(h)
        self.eng.forward_cols(self.recv, x, 1, 0)
        return x

    # ---- inverse: column layout -> row layout (in place on x, or into out with a pointwise factor y)
    def inverse_rows_piece(self, out, i):
        a0, ra = self.pieces[i]
        self.eng.inverse_rows(self.recv, out, a0, ra)

    def _inverse_tail(self, out):
        hs = [self.exchange.start(self.send, self.recv, 1, a0, ra) for a0, ra in self.pieces]
        for i, h in enumerate(hs):
            self.exchange.wait(h)
            self.inverse_rows_piece(out, i)
        return out

    def inverse(self, x):
        self.eng.inverse_cols(x, None, self.send)
        return self._inverse_tail(x)

    # ---- polynomial multiply: row-layout a, b -> row-layout out = a * b (cyclic, length n).
    # a and b are left holding their column-layout forward transforms (unless out aliases them).
    def polymul(self, a, b, out):
        if a is b:  # squaring: one forward, single-vector exchange
            self.forward(a)
        else:
            send2, recv2 = self.pair_buffers()
            hs = []
            for i, (a0, ra) in enumerate(self.pieces):
                self.forward_rows_piece(a, i, 2, 0, send2)
                self.forward_rows_piece(b, i, 2, 1, send2)
                hs.append(self.exchange.start(send2, recv2, 2, a0, ra))
            for h in hs:
                self.exchange.wait(h)
            self.eng.forward_cols(recv2, a, 2, 0)
            self.eng.forward_cols(recv2, b, 2, 1)
        self.eng.inverse_cols(a, b, self.send)
        return self._inverse_tail(out)


class _WholeExchange:
    """Adapter for a plain ``exchange(send, recv)`` callable: whole-chunk all-to-all, one piece."""

    def __init__(self, fn):
        self.fn = fn

    def start(self, send, recv, nvec, row0, nrows):
        self.fn(send, recv)

    def wait(self, handle):
        pass


def piece_views(buf, world: int, nvec: int, r: int, c: int, row0: int, nrows: int):
    """[peer][vec] views of rows [row0, row0 + nrows) of a [G][nvec][r][c] exchange buffer: each a
    contiguous run of nrows * c elements."""
    b = buf.view(world, nvec, r * c, *buf.shape[1:])
    return [[b[g, v, row0 * c:(row0 + nrows) * c] for v in range(nvec)] for g in range(world)]


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


class DistNTT:
    """One rank of a distributed NTT: the fused rank plan + torch.distributed all-to-all (RCCL on GPUs).

    The default process group must be initialised (``nccl`` backend = RCCL on ROCm).  ``forward``
    takes this rank's row-layout share and leaves its column-layout share in place; ``inverse`` the
    reverse.  See module docstring for the layouts.  The all-to-all runs in ``pieces`` row pieces,
    each an asynchronous RCCL all-to-all on the communicator's stream, overlapping the row transforms
    (FourStep).
    """

    # A piece's row transforms must still fill the GPU: every pass of a local transform launches one
    # 1024-element workgroup tile per 1024 elements, and 256 CUs x 4 resident workgroups want several
    # rounds of them.  Measured on one GPU (profiles/r02_pipe/, configs.jsonl): 2^28 over 8 virtual
    # ranks (2^25 per rank) 34.5 -> 33.5 ms with 4 pieces; 2^24 polymul over 8 (2^21 per rank)
    # 6.8 -> 8.0 ms with 4 pieces (half-empty launches).
    MIN_PIECE_ELEMS = 1 << 22

    @classmethod
    def auto_pieces(cls, local_n: int, cap: int = 8) -> int:
        k = 1
        while k < cap and local_n // (2 * k) >= cls.MIN_PIECE_ELEMS:
            k *= 2
        return k

    def __init__(self, field_id: int = 1, log_n: int = 24, limbs64: int = 4, device: Optional[int] = None,
                 group=None, host_exchange: bool = False, pieces: Optional[int] = None):
        """host_exchange: stage the all-to-all through host memory over a gloo group (rehearsing
        several ranks on ONE GPU, where RCCL refuses duplicate devices); never the product path.
        pieces: row pieces of the pipelined exchange (None: auto_pieces of the local share)."""
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
        if pieces is None:  # world 1: no exchange to hide
            pieces = 1 if world == 1 else self.auto_pieces(self.layout.local_n)
        self.fs = FourStep(self.layout, self.engine, self, pieces=pieces)
        self.n = self.layout.n
        self.passes: List[int] = []  # per-transform schedules: see the row / column plans
        # exchange timing (set_profiling): one window per all-to-all, from the first piece's start to
        # the last piece's arrival, as HIP events on the compute stream (so a window that overlaps
        # row transforms of later pieces includes them)
        self._x_windows: Optional[list] = None
        self._x_open: Optional[list] = None

    # RCCL moves < 2 GiB per peer per collective (a 2 GiB chunk arrived half copied,
    # tests/test_gpu_fullsize.py): larger per-peer runs go as several all-to-alls.
    MAX_PEER_BYTES = 1 << 30

    # ---- FourStep exchange interface: rows [row0, row0 + nrows) of every peer chunk
    def start(self, send, recv, nvec, row0, nrows):
        L = self.layout
        if self._x_windows is not None and (self._x_open is None or self._x_open[1] is not None):
            if self._x_open is not None:
                self._x_windows.append(self._x_open)
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            self._x_open = [e0, None]
        sv = piece_views(send, L.world, nvec, L.r, L.c, row0, nrows)
        rv = piece_views(recv, L.world, nvec, L.r, L.c, row0, nrows)
        works = []
        for v in range(nvec):
            ins = [sv[g][v] for g in range(L.world)]
            outs = [rv[g][v] for g in range(L.world)]
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

    def forward(self, t: torch.Tensor) -> torch.Tensor:
        return self.fs.forward(t)

    def inverse(self, t: torch.Tensor) -> torch.Tensor:
        return self.fs.inverse(t)

    def polymul(self, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """Row-layout shares a, b -> row-layout share of c = a * b (cyclic, length n); two all-to-alls."""
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
        """Row-transform launches, then column-transform launches (separate timing rings)."""
        return self.engine.last_launch_ms(0) + self.engine.last_launch_ms(1)


class VirtualRanks:
    """G ranks of the four-step in ONE process on one GPU; the all-to-all is device copies.

    SURVEY §4: validate the distributed decomposition on a single GPU before RCCL.  With ``pieces``
    > 1 the copies of each row piece run on a side stream while the next piece's row transforms run
    (the schedule of FourStep, interleaved over the G ranks).
    """

    def __init__(self, field_id: int, log_n: int, limbs64: int, world: int, device: int = 0, pieces: int = 1):
        self.world = world
        self.engines = [RankPlan(field_id, log_n, limbs64, world, g, device) for g in range(world)]
        self.ranks = [FourStep(e.layout, e, pieces=pieces) for e in self.engines]
        self.layout0 = self.ranks[0].L
        self.pieces = self.ranks[0].pieces
        self.side = torch.cuda.Stream(device=device)

    def _copy_piece(self, sends, recvs, nvec, row0, nrows):
        """Rows [row0, row0 + nrows) of every (src -> dst) chunk, on the side stream after the work
        enqueued so far; returns the event that marks their arrival."""
        L, G = self.layout0, self.world
        ev = torch.cuda.Event()
        ev.record()
        self.side.wait_event(ev)
        with torch.cuda.stream(self.side):
            sv = [piece_views(t, G, nvec, L.r, L.c, row0, nrows) for t in sends]
            rv = [piece_views(t, G, nvec, L.r, L.c, row0, nrows) for t in recvs]
            for dst in range(G):
                for src in range(G):
                    for v in range(nvec):
                        rv[dst][src][v].copy_(sv[src][dst][v])
            done = torch.cuda.Event()
            done.record()
        for t in list(sends) + list(recvs):  # the side stream uses them: keep the caching allocator honest
            t.record_stream(self.side)
        return done

    def empty(self) -> List[torch.Tensor]:
        return [e.empty(self.layout0.local_n) for e in self.engines]

    def fill(self, xs: List[torch.Tensor], kind: str = "random", seed: int = 1):
        for e, t in zip(self.engines, xs):
            e.fill(t, kind, seed)
        return xs

    def forward(self, xs: List[torch.Tensor]):
        evs = []
        for i, (a0, ra) in enumerate(self.pieces):
            for fs, x in zip(self.ranks, xs):
                fs.forward_rows_piece(x, i)
            evs.append(self._copy_piece([fs.send for fs in self.ranks], [fs.recv for fs in self.ranks], 1, a0, ra))
        for ev in evs:
            torch.cuda.current_stream().wait_event(ev)
        for fs, x in zip(self.ranks, xs):
            fs.eng.forward_cols(fs.recv, x, 1, 0)
        return xs

    def _inverse_tail(self, outs):
        evs = [self._copy_piece([fs.send for fs in self.ranks], [fs.recv for fs in self.ranks], 1, a0, ra)
               for a0, ra in self.pieces]
        for i, ev in enumerate(evs):
            torch.cuda.current_stream().wait_event(ev)
            for fs, o in zip(self.ranks, outs):
                fs.inverse_rows_piece(o, i)
        return outs

    def inverse(self, xs: List[torch.Tensor]):
        for fs, x in zip(self.ranks, xs):
            fs.eng.inverse_cols(x, None, fs.send)
        return self._inverse_tail(xs)

    def polymul(self, As: List[torch.Tensor], Bs: List[torch.Tensor], Outs: List[torch.Tensor]):
        if all(a is b for a, b in zip(As, Bs)):
            self.forward(As)
        else:
            pairs = [fs.pair_buffers() for fs in self.ranks]
            sends, recvs = [p[0] for p in pairs], [p[1] for p in pairs]
            evs = []
            for i, (a0, ra) in enumerate(self.pieces):
                for g, fs in enumerate(self.ranks):
                    fs.forward_rows_piece(As[g], i, 2, 0, sends[g])
                    fs.forward_rows_piece(Bs[g], i, 2, 1, sends[g])
                evs.append(self._copy_piece(sends, recvs, 2, a0, ra))
            for ev in evs:
                torch.cuda.current_stream().wait_event(ev)
            for g, fs in enumerate(self.ranks):
                fs.eng.forward_cols(recvs[g], As[g], 2, 0)
                fs.eng.forward_cols(recvs[g], Bs[g], 2, 1)
        for fs, a, b in zip(self.ranks, As, Bs):
            fs.eng.inverse_cols(a, b, fs.send)
        return self._inverse_tail(Outs)


class MultiPlan:
    """Single-process multi-GPU plan over the C ABI (``ntt_mplan_*``, ntt_amd/csrc/ntt_multi.cpp):
    one process drives ``devices`` with the same four-step and layouts as DistNTT, the exchange
    being one grouped RCCL all-to-all.  Shares are torch tensors, ``xs[g]`` on ``devices[g]``.
    """

    def __init__(self, field_id: int = 1, log_n: int = 24, limbs64: int = 4, devices: Optional[List[int]] = None,
                 pieces: Optional[int] = None):
        """pieces: row pieces of the pipelined exchange (None: the plan's default, >= 2^22 elements each)."""
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
        if pieces is not None:
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
