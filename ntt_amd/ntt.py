"""Host-side mirror of the reference's NTT entry points over libntt.so.

Reference interfaces mirrored (tie-pilot-qxw/NTT):

* ``SSIP(x, omega, log_n)``                      — ``src/GZKP-NTT.cu:1452`` (forward, in place,
  natural order, ``long long`` elements, P = 469762049, ``omega`` = the generator ``root`` = 3).
* ``NTT_GZKP(data, length, prime, omega, B, G)``  — ``src/big-num.cu:260`` (256-bit elements,
  ``cgbn_mem_t<256>`` layout, modulus-generic).  ``reverse``/``B``/``G`` are tuning inputs of the
  reference's non-self-sorting schedule and are accepted but unused.
* inverse                                         — ``src/GZKP-NTT.cu:1725-1732``.

Device data are torch tensors on a HIP device (PyTorch is plumbing here: device memory and
streams); every transform runs in the HIP kernels of libntt.so.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, List, Optional, Sequence

import numpy as np
import torch

from . import lib as _L
from .fields import FIELDS, field_params

__all__ = ["NTTPlan", "SSIP", "NTT_GZKP", "to_device", "from_device", "FIELDS"]


def _stream_ptr(stream, device) -> C.c_void_p:
    if stream is None:
        stream = torch.cuda.current_stream(device)
    return C.c_void_p(stream.cuda_stream)


def _u64_array(values: Sequence[int]):
    arr = (C.c_uint64 * len(values))(*[int(v) & ((1 << 64) - 1) for v in values])
    return arr


def int_to_limbs(v: int, limbs64: int) -> List[int]:
    return [(v >> (64 * i)) & ((1 << 64) - 1) for i in range(limbs64)]


def to_device(values: Iterable[int], limbs64: int, device="cuda") -> torch.Tensor:
    """Python ints -> device tensor in the cgbn_mem_t layout (int64 [n, limbs64]; [n] for 1 limb)."""
    vals = list(values)
    if limbs64 == 1:
        host = np.array(vals, dtype=np.int64)
        return torch.from_numpy(host).to(device)
    host = np.zeros((len(vals), limbs64), dtype=np.uint64)
    for j, v in enumerate(vals):
        for i in range(limbs64):
            host[j, i] = (v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF
    return torch.from_numpy(host.view(np.int64)).to(device)


def from_device(t: torch.Tensor) -> List[int]:
    """Device tensor (cgbn_mem_t layout) -> Python ints."""
    host = t.detach().cpu().numpy()
    if host.ndim == 1:
        return [int(v) for v in host]
    u = host.view(np.uint64)
    out = []
    for row in u:
        v = 0
        for i in range(len(row) - 1, -1, -1):
            v = (v << 64) | int(row[i])
        out.append(v)
    return out


BEALTO_FLAGS = {"bellperson": _L.NTT_PLAN_BELLPERSON, "v1": _L.NTT_PLAN_IMPROVED_V1, "v2": _L.NTT_PLAN_IMPROVED_V2,
                "v3": _L.NTT_PLAN_IMPROVED_V3, "v4": _L.NTT_PLAN_IMPROVED_V4}


class NTTPlan:
    """A cached transform plan: twiddle tables and scratch live on the device.

    ``field_id`` selects a built-in field (0 P469762049, 1 BN254 Fr, 2 BLS12-381 Fr); or pass
    ``modulus``/``generator`` ints for any odd prime below 2^(64*limbs64 - 1) with 2^log_n | p - 1
    (big-num.cu's modulus-generic path).
    """

    def __init__(self, field_id: int = 1, log_n: int = 10, limbs64: int = 4, device: int = 0,
                 modulus: Optional[int] = None, generator: Optional[int] = None, twiddle_only: bool = False,
                 montgomery_io: bool = False, stockham: bool = False, gzkp: bool = False,
                 in_place: bool = False, single_launch: bool = False, naive: bool = False,
                 no_swap: bool = False, bealto: str = ""):
        if bealto and bealto not in BEALTO_FLAGS:
            raise ValueError(f"bealto must be one of {sorted(BEALTO_FLAGS)}, not {bealto!r}")
        self._lib = _L.load()
        self.log_n = int(log_n)
        self.n = 1 << self.log_n
        self.limbs64 = int(limbs64)
        self.device = int(device)
        self.field_id = field_id if modulus is None else None
        if modulus is None:
            self.p, self.g = field_params(field_id)
        else:
            self.p, self.g = int(modulus), int(generator)
        h = C.c_void_p()
        flags = (_L.NTT_PLAN_TWIDDLE_ONLY if twiddle_only else 0) | (_L.NTT_PLAN_MONTGOMERY_IO if montgomery_io else 0)
        # stockham: forward transforms on the reference's bellperson-family rival schedule (ntt.h)
        flags |= _L.NTT_PLAN_STOCKHAM if stockham else 0
        # gzkp: the reference's GZKP(B, G) rival schedule (bit reversal + in-place DIT passes)
        flags |= _L.NTT_PLAN_GZKP if gzkp else 0
        # naive: the reference's `naive` rival (bit reversal + one radix-2 round per launch)
        flags |= _L.NTT_PLAN_NAIVE if naive else 0
        # no_swap: the reference's `naive_no_swap` rival (radix-2 Stockham autosort, one round per launch)
        flags |= _L.NTT_PLAN_NO_SWAP if no_swap else 0
        # bealto: the reference's radix-2^deg group-FFT rivals -- "bellperson" (bellperson_baseline /
        # FIELD_radix_fft_revised) or "v1".."v4" (improved_NTT_v1..v4), one k_bealto launch per round
        flags |= BEALTO_FLAGS[bealto] if bealto else 0
        # in_place: no plan scratch, palindromic passes + tile-swap digit reversal (the reference's
        # self-sort-in-place property, GZKP-NTT.cu:1359-1449; ntt.h NTT_PLAN_IN_PLACE)
        flags |= _L.NTT_PLAN_IN_PLACE if in_place else 0
        # single_launch: 3-pass transforms as one persistent launch (BASELINE config 2's single kernel)
        flags |= _L.NTT_PLAN_SINGLE_LAUNCH if single_launch else 0
        self.montgomery_io = bool(montgomery_io)
        if modulus is None:
            st = self._lib.ntt_plan_create_ex(C.byref(h), int(field_id), self.log_n, self.limbs64, self.device, flags)
        else:
            st = self._lib.ntt_plan_create_custom_ex(C.byref(h), _u64_array(int_to_limbs(self.p, self.limbs64)),
                                                     _u64_array(int_to_limbs(self.g, self.limbs64)), self.limbs64,
                                                     self.log_n, self.device, flags)
        _L.check(st, "ntt_plan_create")
        self._h = h
        n = C.c_uint64()
        eb = C.c_uint()
        npass = C.c_uint()
        radix = (C.c_uint * 8)()
        _L.check(self._lib.ntt_plan_info(h, C.byref(n), C.byref(eb), C.byref(npass), radix), "ntt_plan_info")
        self.elem_bytes = eb.value
        self.passes = [radix[i] for i in range(npass.value)]

    # -------------------------------------------------------------------------------- memory
    def empty(self, batch: int = 1) -> torch.Tensor:
        shape = (batch * self.n,) if self.limbs64 == 1 else (batch * self.n, self.limbs64)
        return torch.empty(shape, dtype=torch.int64, device=f"cuda:{self.device}")

    def _check_tensor(self, t: torch.Tensor, batch: int = 1) -> None:
        if not t.is_cuda:
            raise ValueError("NTT data must be a device (HIP) tensor")
        if not t.is_contiguous() or t.dtype != torch.int64:
            raise ValueError("NTT data must be a contiguous int64 tensor in the cgbn_mem_t layout")
        if t.numel() * 8 != batch * self.n * self.elem_bytes:
            raise ValueError(f"expected {batch * self.n} elements of {self.elem_bytes} bytes")
        if t.device.index != self.device:
            raise ValueError(f"tensor on {t.device}, plan on cuda:{self.device}")

    # -------------------------------------------------------------------------------- transforms
    def forward(self, t: torch.Tensor, stream=None) -> torch.Tensor:
        self._check_tensor(t)
        _L.check(self._lib.ntt_forward(self._h, C.c_void_p(t.data_ptr()), _stream_ptr(stream, t.device)),
                 "ntt_forward")
        return t

    def inverse(self, t: torch.Tensor, stream=None) -> torch.Tensor:
        self._check_tensor(t)
        _L.check(self._lib.ntt_inverse(self._h, C.c_void_p(t.data_ptr()), _stream_ptr(stream, t.device)),
                 "ntt_inverse")
        return t

    def device_status(self) -> int:
        """ntt_plan_device_status: bit 0 = a watchdog gave up (single launch / fused in-place digit
        reversal; until this clears it, every call on the plan raises NTTError NTT_ERR_DEVICE); with
        the checked build (libntt_debug.so) 0x100 bounds, 0x200 non-canonical input, 0x400 lazy bound,
        0x800 non-canonical output.  Blocking (synchronises the device); clears the report."""
        v = C.c_uint()
        _L.check(self._lib.ntt_plan_device_status(self._h, C.byref(v)), "ntt_plan_device_status")
        return v.value

    def set_watchdog(self, spins: int = 1 << 21) -> None:
        """ntt_plan_set_watchdog: poll limit of the plan's inter-workgroup waits (0 = give up at once,
        a test hook for the NTT_ERR_DEVICE path)."""
        _L.check(self._lib.ntt_plan_set_watchdog(self._h, int(spins)), "ntt_plan_set_watchdog")

    def count_noncanonical(self, t: torch.Tensor, stream=None) -> int:
        """Number of elements of t that are not < p (the transforms' input contract); blocking."""
        if t.device.type != "cuda" or not t.is_contiguous() or t.dtype != torch.int64:
            raise ValueError("expected a contiguous int64 device tensor in the element layout")
        count = t.numel() if self.limbs64 == 1 else t.numel() // self.limbs64
        bad = C.c_uint64()
        _L.check(self._lib.ntt_count_noncanonical(self._h, C.c_void_p(t.data_ptr()), count, C.byref(bad),
                                                  _stream_ptr(stream, t.device)), "ntt_count_noncanonical")
        return bad.value

    def forward_batch(self, t: torch.Tensor, batch: int, stream=None) -> torch.Tensor:
        self._check_tensor(t, batch)
        _L.check(self._lib.ntt_forward_batch(self._h, C.c_void_p(t.data_ptr()), int(batch),
                                             _stream_ptr(stream, t.device)), "ntt_forward_batch")
        return t

    def inverse_batch(self, t: torch.Tensor, batch: int, stream=None) -> torch.Tensor:
        self._check_tensor(t, batch)
        _L.check(self._lib.ntt_inverse_batch(self._h, C.c_void_p(t.data_ptr()), int(batch),
                                             _stream_ptr(stream, t.device)), "ntt_inverse_batch")
        return t

    def forward_coset(self, t: torch.Tensor, shift: int, stream=None) -> torch.Tensor:
        """Evaluations on the coset shift*<w>: X_k = sum_j x_j (shift w^k)^j (low-degree extension)."""
        self._check_tensor(t)
        _L.check(self._lib.ntt_forward_coset(self._h, C.c_void_p(t.data_ptr()),
                                             _u64_array(int_to_limbs(int(shift), self.limbs64)),
                                             _stream_ptr(stream, t.device)), "ntt_forward_coset")
        return t

    def inverse_coset(self, t: torch.Tensor, shift: int, stream=None) -> torch.Tensor:
        """Interpolation from the coset shift*<w>: x_j = shift^-j INTT(X)_j."""
        self._check_tensor(t)
        _L.check(self._lib.ntt_inverse_coset(self._h, C.c_void_p(t.data_ptr()),
                                             _u64_array(int_to_limbs(int(shift), self.limbs64)),
                                             _stream_ptr(stream, t.device)), "ntt_inverse_coset")
        return t

    def pointwise_mul(self, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, stream=None) -> torch.Tensor:
        for t in (a, b, out):
            self._check_tensor(t)
        _L.check(self._lib.ntt_pointwise_mul(self._h, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()),
                                             C.c_void_p(out.data_ptr()), _stream_ptr(stream, a.device)),
                 "ntt_pointwise_mul")
        return out

    def polymul(self, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, stream=None) -> torch.Tensor:
        for t in (a, b, out):
            self._check_tensor(t)
        _L.check(self._lib.ntt_polymul(self._h, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()),
                                       C.c_void_p(out.data_ptr()), _stream_ptr(stream, a.device)), "ntt_polymul")
        return out

    def inverse_pointwise_batch(self, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, batch: int,
                                stream=None) -> torch.Tensor:
        """out = INTT(a * b) over `batch` transforms (a, b already forward-transformed)."""
        for t in (a, b, out):
            self._check_tensor(t, batch)
        _L.check(self._lib.ntt_inverse_pointwise_batch(self._h, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()),
                                                       C.c_void_p(out.data_ptr()), int(batch),
                                                       _stream_ptr(stream, a.device)), "ntt_inverse_pointwise_batch")
        return out

    def fill(self, t: torch.Tensor, kind: str = "random", seed: int = 1, stream=None) -> torch.Tensor:
        """SURVEY §8d synthetic inputs on the device: 'iota' (x_j = j) or 'random' (SplitMix64)."""
        self._check_tensor(t)
        k = {"iota": 0, "random": 1}[kind]
        _L.check(self._lib.ntt_fill(self._h, C.c_void_p(t.data_ptr()), k, int(seed), _stream_ptr(stream, t.device)),
                 "ntt_fill")
        return t

    def fill_map(self, t: torch.Tensor, kind: str, seed: int, row0: int, log_inner: int, log_stride: int,
                 stream=None) -> torch.Tensor:
        """Local element i <- synthetic value of global j = row0 + (i >> log_inner) + ((i & m) << log_stride)."""
        count = t.numel() * 8 // self.elem_bytes
        k = {"iota": 0, "random": 1}[kind]
        _L.check(self._lib.ntt_fill_map(self._h, C.c_void_p(t.data_ptr()), count, k, int(seed), int(row0),
                                        int(log_inner), int(log_stride), _stream_ptr(stream, t.device)),
                 "ntt_fill_map")
        return t

    def twiddle_pack(self, src: torch.Tensor, dst: torch.Tensor, log_rows: int, log_row_len: int, log_block: int,
                     row0: int, inverse: bool = False, stream=None, peer_stride: Optional[int] = None) -> torch.Tensor:
        """dst[q * peer_stride + a * bw + b % bw] = src[a][b] * w_n^(+-(row0 + a) * b), q = b >> log_block
        (four-step twiddle + pack; peer_stride defaults to the dense 2^(log_rows + log_block))."""
        ps = (1 << (log_rows + log_block)) if peer_stride is None else int(peer_stride)
        _L.check(self._lib.ntt_twiddle_pack_ex(self._h, C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                               int(log_rows), int(log_row_len), int(log_block), int(row0),
                                               int(bool(inverse)), ps, _stream_ptr(stream, src.device)),
                 "ntt_twiddle_pack_ex")
        return dst

    def transpose(self, src: torch.Tensor, dst: torch.Tensor, log_rows: int, log_cols: int, stream=None,
                  log_block_rows: Optional[int] = None, block_stride: Optional[int] = None):
        """dst[c][r] = src row r, column c; source rows in blocks of 2^log_block_rows starting every
        block_stride elements (default: one dense [rows][cols] matrix)."""
        lb = log_rows if log_block_rows is None else int(log_block_rows)
        bs = (1 << (lb + log_cols)) if block_stride is None else int(block_stride)
        _L.check(self._lib.ntt_transpose_ex(self._h, C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                            int(log_rows), int(log_cols), lb, bs, _stream_ptr(stream, src.device)),
                 "ntt_transpose_ex")
        return dst

    def set_profiling(self, enable: bool = True) -> None:
        _L.check(self._lib.ntt_plan_set_profiling(self._h, int(bool(enable))), "ntt_plan_set_profiling")

    def last_launch_ms(self) -> List[float]:
        """Kernel durations (ms, HIP events on the launch stream) of the most recent transform."""
        buf = (C.c_float * 16)()
        k = C.c_uint()
        _L.check(self._lib.ntt_plan_last_launch_ms(self._h, buf, 16, C.byref(k)), "ntt_plan_last_launch_ms")
        return [buf[i] for i in range(k.value)]

    def last_launch_labels(self) -> List[str]:
        """Labels of the same launches (ntt.h ntt_plan_last_launch_labels: c8, c8s, f8, ...)."""
        buf = C.create_string_buffer(256)
        _L.check(self._lib.ntt_plan_last_launch_labels(self._h, buf, 256), "ntt_plan_last_launch_labels")
        v = buf.value.decode()
        return v.split(",") if v else []

    def profile_group(self) -> None:
        """Group mode (ntt.h ntt_plan_profile_group): later transforms join one record until the next call."""
        _L.check(self._lib.ntt_plan_profile_group(self._h), "ntt_plan_profile_group")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.ntt_plan_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown ordering
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------------------------ shims
def SSIP(x: torch.Tensor, omega: int = 3, log_n: Optional[int] = None) -> torch.Tensor:
    """Reference ``SSIP(long long* x, long long omega, uint log_n)`` (GZKP-NTT.cu:1452): forward NTT
    over P = 469762049 in place on a device int64 tensor; blocking like the reference."""
    lib = _L.load()
    if log_n is None:
        log_n = int(x.numel()).bit_length() - 1
    if x.dtype != torch.int64 or not x.is_cuda or x.numel() != (1 << log_n):
        raise ValueError("SSIP expects a device int64 tensor of 2^log_n elements")
    with torch.cuda.device(x.device):
        lib.SSIP(C.c_void_p(x.data_ptr()), int(omega), int(log_n))
    _L.check(lib.ntt_last_error(), "SSIP")
    return x


def NTT_GZKP(data: torch.Tensor, length: int, prime: int, omega: int, B: int = 5, G: int = 8) -> torch.Tensor:
    """Reference ``NTT_GZKP<8,256>(data, len, reverse, reverse_len, prime, omega, B, G)``
    (big-num.cu:260): 256-bit elements, modulus-generic, in place, blocking."""
    lib = _L.load()
    if data.dtype != torch.int64 or not data.is_cuda or data.numel() != 4 * length:
        raise ValueError("NTT_GZKP expects a device int64 tensor [len, 4] (cgbn_mem_t<256>)")
    p32 = (C.c_uint32 * 8)(*[(prime >> (32 * i)) & 0xFFFFFFFF for i in range(8)])
    g32 = (C.c_uint32 * 8)(*[(omega >> (32 * i)) & 0xFFFFFFFF for i in range(8)])
    with torch.cuda.device(data.device):
        st = lib.NTT_GZKP_256(C.c_void_p(data.data_ptr()), int(length), None, 0, p32, g32, int(B), int(G))
    _L.check(st, "NTT_GZKP")
    return data
