"""Multi-GPU NTT: four-step decomposition with one all-to-all.

n = n1 * n2, j = j1 + n1*j2, k = k2 + n2*k1:

    X[k2 + n2 k1] = sum_j1 w_n1^(j1 k1) * w_n^(j1 k2) * sum_j2 w_n2^(j2 k2) x[j1 + n1 j2]

Rank g of G (one process per GPU, ``torch.distributed`` over RCCL) owns

* input, "row layout":    rows j1 in [g r, (g+1) r), r = n1/G; local [r][n2], element (a, j2) = x[g r + a + n1 j2]
* output, "column layout": cols k2 in [g c, (g+1) c), c = n2/G; local [c][n1], element (kc, k1) = X[g c + kc + n2 k1]

Forward = batched n2-point NTTs of the local rows (libntt) -> twiddle w_n^(j1 k2) fused with the pack
into per-peer chunks (libntt ntt_twiddle_pack) -> ONE all-to-all (RCCL; each peer chunk r*c elements)
-> local transpose (libntt) -> batched n1-point NTTs (libntt).  The inverse mirrors it (column layout
in, row layout out), so forward/inverse/pointwise products (polynomial multiply) never leave the
distributed layouts.  Gathering to natural order is a separate, test-only helper.

The reference has no multi-GPU code at all (no NCCL/MPI); this is new.
The orchestration (FourStep) is engine- and transport-agnostic so the same code runs with the
HIP engine over RCCL on GPUs, with G "virtual ranks" in one process on one GPU (exchange =
device copies), and with a CPU test engine over gloo.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional

import torch


@dataclass
class Layout:
    log_n: int
    world: int
    rank: int

    def __post_init__(self):
        if self.world < 1 or self.world & (self.world - 1):
            raise ValueError("world size must be a power of two")
        self.log_g = self.world.bit_length() - 1
        self.log_n1 = (self.log_n + 1) // 2
        self.log_n2 = self.log_n // 2
        if self.log_g > self.log_n2:
            raise ValueError(f"2^{self.log_n} is too small to split over {self.world} ranks")
        self.log_r = self.log_n1 - self.log_g  # local rows (row layout)
        self.log_c = self.log_n2 - self.log_g  # local columns (column layout)
        self.n = 1 << self.log_n
        self.n1, self.n2 = 1 << self.log_n1, 1 << self.log_n2
        self.r, self.c = 1 << self.log_r, 1 << self.log_c
        self.local_n = self.n >> self.log_g

    # global index of local element i (tests / fills)
    def row_global(self, i: int) -> int:
        a, j2 = i >> self.log_n2, i & (self.n2 - 1)
        return self.rank * self.r + a + self.n1 * j2

    def col_global(self, i: int) -> int:
        kc, k1 = i >> self.log_n1, i & (self.n1 - 1)
        return self.rank * self.c + kc + self.n2 * k1


class FourStep:
    """Per-rank four-step schedule over an engine (local compute) and an exchange (all-to-all).

    Engine interface: ``rows_forward/rows_inverse(t, batch)`` (batched n2-point NTTs),
    ``cols_forward/cols_inverse(t, batch)`` (batched n1-point NTTs), ``twiddle_pack(src, dst,
    log_rows, log_len, log_block, row0, inverse)``, ``transpose(src, dst, log_rows, log_cols)``,
    ``empty(count)``.  Exchange: ``exchange(send, recv)`` = all-to-all of equal contiguous chunks.
    """

    def __init__(self, layout: Layout, engine, exchange: Optional[Callable] = None):
        self.L = layout
        self.eng = engine
        self.exchange = exchange
        self.send = engine.empty(layout.local_n)
        self.recv = engine.empty(layout.local_n)

    # ---- forward: row layout -> column layout (in place on x)
    def forward_phase1(self, x):
        L = self.L
        self.eng.rows_forward(x, L.r)
        self.eng.twiddle_pack(x, self.send, L.log_r, L.log_n2, L.log_c, L.rank * L.r, False)

    def forward_phase2(self, x):
        L = self.L
        self.eng.transpose(self.recv, x, L.log_n1, L.log_c)  # recv = [G][r][c] = [n1][c]
        self.eng.cols_forward(x, L.c)

    def forward(self, x):
        self.forward_phase1(x)
        self.exchange(self.send, self.recv)
        self.forward_phase2(x)
        return x

    # ---- inverse: column layout -> row layout (in place on x)
    def inverse_phase1(self, x):
        L = self.L
        self.eng.cols_inverse(x, L.c)
        self.eng.twiddle_pack(x, self.send, L.log_c, L.log_n1, L.log_r, L.rank * L.c, True)

    def inverse_phase2(self, x):
        L = self.L
        self.eng.transpose(self.recv, x, L.log_n2, L.log_r)  # recv = [G][c][r] = [n2][r]
        self.eng.rows_inverse(x, L.r)

    def inverse(self, x):
        self.inverse_phase1(x)
        self.exchange(self.send, self.recv)
        self.inverse_phase2(x)
        return x


class HipEngine:
    """Local steps on one GPU through libntt (the product path)."""

    def __init__(self, field_id: int, log_n: int, limbs64: int, world: int, device: int):
        from .ntt import NTTPlan
        L = Layout(log_n, world, 0)
        self.rows = NTTPlan(field_id, L.log_n2, limbs64, device)
        self.cols = self.rows if L.log_n1 == L.log_n2 else NTTPlan(field_id, L.log_n1, limbs64, device)
        self.tw = NTTPlan(field_id, log_n, limbs64, device, twiddle_only=True)
        self.limbs64 = limbs64
        self.device = device

    def empty(self, count: int) -> torch.Tensor:
        shape = (count,) if self.limbs64 == 1 else (count, self.limbs64)
        return torch.empty(shape, dtype=torch.int64, device=f"cuda:{self.device}")

    def rows_forward(self, t, batch):
        self.rows.forward_batch(t, batch)

    def rows_inverse(self, t, batch):
        self.rows.inverse_batch(t, batch)

    def cols_forward(self, t, batch):
        self.cols.forward_batch(t, batch)

    def cols_inverse(self, t, batch):
        self.cols.inverse_batch(t, batch)

    def twiddle_pack(self, src, dst, log_rows, log_len, log_block, row0, inverse):
        self.tw.twiddle_pack(src, dst, log_rows, log_len, log_block, row0, inverse)

    def transpose(self, src, dst, log_rows, log_cols):
        self.tw.transpose(src, dst, log_rows, log_cols)

    def plans(self):
        return [self.rows] if self.cols is self.rows else [self.rows, self.cols]


class DistNTT:
    """One rank of a distributed NTT: HIP engine + torch.distributed all-to-all (RCCL on GPUs).

    The default process group must be initialised (``nccl`` backend = RCCL on ROCm).  ``forward``
    takes this rank's row-layout share and leaves its column-layout share in place; ``inverse`` the
    reverse.  See module docstring for the layouts.
    """

    def __init__(self, field_id: int = 1, log_n: int = 24, limbs64: int = 4, device: Optional[int] = None,
                 group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        if device is None:
            device = torch.cuda.current_device()
        self.device = device
        self.field_id, self.log_n, self.limbs64 = field_id, log_n, limbs64
        self.layout = Layout(log_n, world, rank)
        self.engine = HipEngine(field_id, log_n, limbs64, world, device)
        self.fs = FourStep(self.layout, self.engine, self._exchange)
        self.n = self.layout.n
        self.passes = self.engine.rows.passes

    def _exchange(self, send, recv):
        self.dist.all_to_all_single(recv.view(-1), send.view(-1), group=self.group)

    def empty(self) -> torch.Tensor:
        return self.engine.empty(self.layout.local_n)

    def fill(self, t: torch.Tensor, kind: str = "random", seed: int = 1) -> torch.Tensor:
        """This rank's row-layout share of the global synthetic vector (same values as NTTPlan.fill)."""
        L = self.layout
        self.engine.tw.fill_map(t, kind, seed, L.rank * L.r, L.log_n2, L.log_n1)
        return t

    def forward(self, t: torch.Tensor) -> torch.Tensor:
        return self.fs.forward(t)

    def inverse(self, t: torch.Tensor) -> torch.Tensor:
        return self.fs.inverse(t)

    def set_profiling(self, enable: bool = True) -> None:
        for p in self.engine.plans():
            p.set_profiling(enable)

    def last_launch_ms(self) -> List[float]:
        out: List[float] = []
        for p in self.engine.plans():
            out += p.last_launch_ms()
        return out


class VirtualRanks:
    """G ranks of the four-step in ONE process on one GPU; the all-to-all is device copies.

    SURVEY §4: validate the distributed decomposition on a single GPU before RCCL.
    """

    def __init__(self, field_id: int, log_n: int, limbs64: int, world: int, device: int = 0):
        self.world = world
        self.engine = HipEngine(field_id, log_n, limbs64, world, device)
        self.ranks = [FourStep(Layout(log_n, world, g), self.engine) for g in range(world)]
        self.layout0 = self.ranks[0].L

    def _exchange_all(self):
        G = self.world
        chunk = self.layout0.local_n // G
        for dst in range(G):
            for src in range(G):
                self.ranks[dst].recv[src * chunk:(src + 1) * chunk].copy_(
                    self.ranks[src].send[dst * chunk:(dst + 1) * chunk])

    def empty(self) -> List[torch.Tensor]:
        return [self.engine.empty(self.layout0.local_n) for _ in range(self.world)]

    def fill(self, xs: List[torch.Tensor], kind: str = "random", seed: int = 1):
        for g, t in enumerate(xs):
            L = self.ranks[g].L
            self.engine.tw.fill_map(t, kind, seed, g * L.r, L.log_n2, L.log_n1)
        return xs

    def forward(self, xs: List[torch.Tensor]):
        for fs, x in zip(self.ranks, xs):
            fs.forward_phase1(x)
        self._exchange_all()
        for fs, x in zip(self.ranks, xs):
            fs.forward_phase2(x)
        return xs

    def inverse(self, xs: List[torch.Tensor]):
        for fs, x in zip(self.ranks, xs):
            fs.inverse_phase1(x)
        self._exchange_all()
        for fs, x in zip(self.ranks, xs):
            fs.inverse_phase2(x)
        return xs


class MultiPlan:
    """Single-process multi-GPU plan over the C ABI (``ntt_mplan_*``, ntt_amd/csrc/ntt_multi.cpp):
    one process drives ``devices`` with the same four-step and layouts as DistNTT, the exchange
    being one grouped RCCL all-to-all.  Shares are torch tensors, ``xs[g]`` on ``devices[g]``.
    """

    def __init__(self, field_id: int = 1, log_n: int = 24, limbs64: int = 4, devices: Optional[List[int]] = None):
        import ctypes as C
        from . import lib as _L
        self._C, self._L = C, _L
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
        self.layouts = [Layout(log_n, len(self.devices), g) for g in range(len(self.devices))]

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            self.lib.ntt_mplan_destroy(h)
            self.handle = None

    def empty(self) -> List[torch.Tensor]:
        shape = (self.local_n,) if self.limbs64 == 1 else (self.local_n, self.limbs64)
        return [torch.empty(shape, dtype=torch.int64, device=f"cuda:{d}") for d in self.devices]

    def _ptrs(self, xs):
        C = self._C
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
