"""Config C1 plumbing: the reference's Python helpers, restated (no GPU).

* ``datapath_map(lgp)``       — the write-index map printed by ``src/datapath_demo.py:4-39``
  (``draw_data_flow``) for the bellperson radix kernel ``FIELD_radix_fft`` (GZKP-NTT.cu:324-386) at
  n = 4096, deg = 4: for each of the 256 blocks, the 16 output indices its 8 threads write.
* ``twiddle_exponents(target, origin, omega, p)`` — ``src/twiddlecheck.py:1-15``: for each j the
  exponents i < 256 with origin[j] * omega^i == target[j] (mod p).
* ``cpu_ntt_c1(log_n=12)`` — the C1 CPU transform (2^12 over BN254 Fr) through the same
  definition, used as the plumbing self-check.

These are pure-Python product helpers (the reference's own CPU path is Python here), separate from
the test oracle.
"""
from __future__ import annotations

from typing import List, Sequence

from .fields import BN254_FR, P469762049


def datapath_map(lgp: int, deg: int = 4, n: int = 4096) -> List[List[int]]:
    """Rows of (i*p + y, p*(i+counth) + y) pairs exactly as datapath_demo.py prints them."""
    blockdim = 2 ** deg // 2
    rows = []
    for blockid in range(n // (blockdim * 2)):
        row: List[int] = []
        for threadid in range(blockdim):
            lid, lsize, index = threadid, blockdim, blockid
            p = 1 << lgp
            k = index & (p - 1)
            count = 1 << deg
            counth = count >> 1
            counts = count // lsize * lid
            counte = counts + count // lsize
            y = ((index - k) << deg) + k
            for i in range(counts // 2, counte // 2):
                row.extend((i * p + y, p * (i + counth) + y))
        rows.append(row)
    return rows


def format_datapath_map(rows: Sequence[Sequence[int]]) -> str:
    """Same text as the reference's stdout (space-separated pairs, ' ' + newline per block)."""
    return "".join("".join(f"{v} " for v in row) + " \n" for row in rows)


def twiddle_exponents(target: Sequence[int], origin: Sequence[int], omega: int = 338628632,
                      p: int = P469762049, order: int = 256) -> List[int]:
    """All i < order with origin[j]*omega^i == target[j] (mod p), in j-major order."""
    powers = [pow(omega, i, p) for i in range(order)]
    out: List[int] = []
    for j in range(len(origin)):
        for i in range(order):
            if origin[j] * powers[i] % p == target[j]:
                out.append(i)
    return out


def cpu_ntt(x: Sequence[int], p: int, g: int) -> List[int]:
    """Natural-order forward NTT (radix-2 DIF + bit reversal) on the host CPU."""
    n = len(x)
    L = n.bit_length() - 1
    a = [v % p for v in x]
    m = n
    while m > 1:
        h = m >> 1
        wm = pow(g, (p - 1) // m, p)
        for start in range(0, n, m):
            w = 1
            for j in range(h):
                u, v = a[start + j], a[start + j + h]
                a[start + j] = (u + v) % p
                a[start + j + h] = (u - v) * w % p
                w = w * wm % p
        m = h
    out = [0] * n
    for i in range(n):
        r = int(format(i, f"0{L}b")[::-1], 2) if L else 0
        out[r] = a[i]
    return out


def cpu_ntt_c1(log_n: int = 12) -> List[int]:
    """Config C1: 2^12 forward NTT over BN254 Fr of x_j = j on the CPU."""
    return cpu_ntt(list(range(1 << log_n)), BN254_FR, 5)
