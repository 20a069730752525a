"""CPU oracle for the NTT hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it.  It restates, in plain Python big integers, the
reference's (tie-pilot-qxw/NTT) definition of the transform:

* ``ntt_dit``      — ``NTT`` in ``src/GZKP-NTT.cu:30-48`` (bit-reverse, then radix-2 DIT with
                     ``gap = qpow(omega, (P-1)/(stride<<1))``);  the same definition is used by
                     ``src/big-num.cu:37-55`` and ``src/self-sort-in-place.cu:32-51``.
* ``ssip_pro``     — ``NTT_pro1`` + ``NTT_pro2`` in ``src/self-sort-in-place.cu:79-128`` (the
                     self-sort-in-place dataflow: DIF on the high half of the bits, then mirror-pair
                     DIF on the low half, natural order in and out).
* ``intt``         — the (commented-out) inverse recipe of ``src/GZKP-NTT.cu:1725-1732``: forward
                     with ``inv(root)``, then multiply by ``inv(len)``.
* ``kat_xj``       — closed form for the reference's own input ``x_j = j`` (``GZKP-NTT.cu:1587``):
                     ``X_0 = n(n-1)/2``, ``X_k = n / (w^k - 1)``.
* ``four_step``    — the multi-GPU row/column decomposition, used to check layouts.
* ``coset_ntt`` / ``coset_intt`` / ``kat_coset_xj`` — the coset (low-degree-extension) transform of
                     SURVEY §8f.3, which the reference does not have: evaluations on c<w>,
                     ``X_k = sum_j x_j (c w^k)^j``; pinned by ``dft_direct`` and a closed form for
                     ``x_j = j`` (parity unpinned by the reference itself).
* ``to_mont`` / ``from_mont`` — CGBN's Montgomery domain ``x R mod p``, ``R = 2^(64 limbs64)``
                     (``bn2mont`` / ``mont2bn``, ``impl_cuda.cu:980-1024``), for the Montgomery-form I/O flag.

Parity pins (see tests/test_oracle.py): the closed-form KAT, the reference-run 2^26 outputs recorded
in SURVEY.md §0.3, the twiddle constant hard-coded in ``src/twiddlecheck.py:11``, and golden vectors
captured from the reference's own Python (``tests/golden/make_golden.py``).
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

# ----------------------------------------------------------------------------- fields
P469762049 = 469762049  # GZKP-NTT.cu:7 (the comment "29 * 2^57 + 1" there is wrong: 7*2^26+1)
BN254_FR = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
BLS12_381_FR = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

# field id -> (modulus, multiplicative generator).  root = 3 for P is GZKP-NTT.cu:8.
FIELDS = {
    0: (P469762049, 3),
    1: (BN254_FR, 5),
    2: (BLS12_381_FR, 7),
}
FIELD_NAMES = {0: "P469762049", 1: "BN254_FR", 2: "BLS12_381_FR"}


def two_adicity(p: int) -> int:
    v, s = p - 1, 0
    while v % 2 == 0:
        v //= 2
        s += 1
    return s


def root_of_unity(p: int, g: int, n: int) -> int:
    """omega_n = g^((p-1)/n): GZKP-NTT.cu:1462 (``omega = qpow(omega, (P-1)/n)``), big-num.cu:292-296."""
    assert (p - 1) % n == 0, "n must divide p-1"
    return pow(g, (p - 1) // n, p)


# ----------------------------------------------------------------------------- vectors
MASK64 = (1 << 64) - 1


def splitmix64(c: int) -> int:
    """Stateless SplitMix64 of a 64-bit counter (SURVEY §8d input generator).

    z = c + 0x9E3779B97F4A7C15; z = (z ^ z>>30) * 0xBF58476D1CE4E5B9; z = (z ^ z>>27) * 0x94D049BB133111EB;
    return z ^ z>>31   (all mod 2^64).  The GPU generator (ntt_fill_random) computes the same.
    """
    z = (c + 0x9E3779B97F4A7C15) & MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def top_mask_bits(field_id: int) -> int:
    """Bits kept in the top 64-bit limb so that every generated value is < p without rejection."""
    return {0: 28, 1: 61, 2: 62}[field_id]


def random_vector(field_id: int, n: int, seed: int) -> List[int]:
    """Vector B of SURVEY §8d: limb_i = SplitMix64(seed*2^32 + 4j + i), top limb masked.

    For P (a 1-limb field) only limb 0 is drawn and masked to 28 bits.
    """
    out = []
    if field_id == 0:
        m = (1 << 28) - 1
        for j in range(n):
            out.append(splitmix64((seed << 32) + 4 * j) & m)
        return out
    tm = (1 << top_mask_bits(field_id)) - 1
    for j in range(n):
        v = 0
        for i in range(4):
            limb = splitmix64((seed << 32) + 4 * j + i)
            if i == 3:
                limb &= tm
            v |= limb << (64 * i)
        out.append(v)
    return out


def iota_vector(n: int) -> List[int]:
    """Vector A: x_j = j, the reference's own input (GZKP-NTT.cu:1587, big-num.cu:400)."""
    return list(range(n))


# ----------------------------------------------------------------------------- transforms
def bitrev_table(log_n: int) -> List[int]:
    """reverse[i] = (reverse[i>>1]>>1) | ((i&1) << (bits-1))  — GZKP-NTT.cu:1580-1582."""
    n = 1 << log_n
    rev = [0] * n
    for i in range(1, n):
        rev[i] = (rev[i >> 1] >> 1) | ((i & 1) << (log_n - 1))
    return rev


def ntt_dit(x: Sequence[int], p: int, g: int) -> List[int]:
    """Forward NTT, natural order in and out.  Restates GZKP-NTT.cu:30-48.

    ``g`` is the field generator (the reference passes ``root``); stage twiddles are
    ``gap = g^((p-1)/(2*stride))`` exactly as the reference computes them.
    """
    n = len(x)
    log_n = n.bit_length() - 1
    assert n == 1 << log_n
    data = [v % p for v in x]
    if n == 1:
        return data
    rev = bitrev_table(log_n)
    for i in range(n):
        if i < rev[i]:
            data[i], data[rev[i]] = data[rev[i]], data[i]
    stride = 1
    while stride < n:
        gap = pow(g, (p - 1) // (stride << 1), p)
        for start in range(0, n, stride << 1):
            w = 1
            for off in range(stride):
                a = data[start + off]
                b = w * data[start + off + stride] % p
                data[start + off] = (a + b) % p
                data[start + off + stride] = (a - b) % p
                w = gap * w % p
        stride <<= 1
    return data


def ssip_pro(x: Sequence[int], p: int, g: int) -> List[int]:
    """Self-sort-in-place dataflow, NTT_pro1 + NTT_pro2 (self-sort-in-place.cu:79-128).

    Produces natural-order output without any bit-reversal pass; checked against ``ntt_dit``.
    """
    n = len(x)
    L = n.bit_length() - 1
    data = [v % p for v in x]
    # NTT_pro1: DIF rounds over the high bits, i = L .. L/2+1
    for i in range(L, L // 2, -1):
        stride = 1 << (i - 1)
        gap = pow(g, (p - 1) // (stride << 1), p)
        for start in range(0, n, stride << 1):
            w = 1
            for off in range(stride):
                a, b = data[start + off], data[start + off + stride]
                data[start + off] = (a + b) % p
                data[start + off + stride] = (a - b) % p * w % p
                w = gap * w % p
    # NTT_pro2: mirror-pair rounds over the low bits, i = L/2 .. 1
    for i in range(L // 2, 0, -1):
        stride = 1 << (i - 1)
        pair_stride = 1 << (L - i)
        gap = pow(g, (p - 1) // (stride << 1), p)
        for start in range(0, n, pair_stride << 1):
            for off0 in range(0, pair_stride, stride << 1):
                w = 1
                for off in range(stride):
                    o = start + off0 + off
                    a, b = data[o], data[o + stride]
                    c, d = data[o + pair_stride], data[o + pair_stride + stride]
                    data[o] = (a + b) % p
                    data[o + stride] = (c + d) % p
                    data[o + pair_stride] = (a - b) % p * w % p
                    data[o + pair_stride + stride] = (c - d) % p * w % p
                    w = gap * w % p
    return data


def intt(X: Sequence[int], p: int, g: int) -> List[int]:
    """Inverse: forward with inv(root), then scale by inv(n) — GZKP-NTT.cu:1725-1732."""
    n = len(X)
    ginv = pow(g, p - 2, p)
    y = ntt_dit(X, p, ginv)
    ninv = pow(n, p - 2, p)
    return [v * ninv % p for v in y]


def dft_direct(x: Sequence[int], p: int, w: int) -> List[int]:
    """O(n^2) definition X_k = sum_j x_j w^(jk) (small n only)."""
    n = len(x)
    return [sum(x[j] * pow(w, j * k, p) for j in range(n)) % p for k in range(n)]


def kat_xj(n: int, p: int, g: int, k: int) -> int:
    """Closed form of NTT(x_j = j) at output k."""
    if k == 0:
        return n * (n - 1) // 2 % p
    w = root_of_unity(p, g, n)
    return n * pow((pow(w, k, p) - 1) % p, p - 2, p) % p


def coset_ntt(x: Sequence[int], p: int, g: int, c: int) -> List[int]:
    """X_k = sum_j x_j (c w^k)^j = NTT(x_j c^j) (evaluations on the coset c<w>)."""
    return ntt_dit([v * pow(c, j, p) % p for j, v in enumerate(x)], p, g)


def coset_intt(X: Sequence[int], p: int, g: int, c: int) -> List[int]:
    """Inverse of coset_ntt: x_j = c^-j INTT(X)_j."""
    ci = pow(c, p - 2, p)
    return [v * pow(ci, j, p) % p for j, v in enumerate(intt(X, p, g))]


def kat_coset_xj(n: int, p: int, g: int, c: int, k: int) -> int:
    """Closed form of coset_ntt(x_j = j) at output k: sum_{j<n} j z^j with z = c w^k, z^n = c^n:
    z (1 - n z^(n-1) + (n-1) z^n) / (1 - z)^2  (z != 1)."""
    w = root_of_unity(p, g, n)
    z = c * pow(w, k, p) % p
    if z == 1:
        return n * (n - 1) // 2 % p
    num = z * (1 - n * pow(z, n - 1, p) + (n - 1) * pow(z, n, p)) % p
    return num * pow((1 - z) ** 2 % p, p - 2, p) % p


def to_mont(v: int, p: int, limbs64: int) -> int:
    return v * pow(2, 64 * limbs64, p) % p


def from_mont(v: int, p: int, limbs64: int) -> int:
    return v * pow(pow(2, 64 * limbs64, p), p - 2, p) % p


def four_step(x: Sequence[int], p: int, g: int, n1: int, n2: int) -> List[int]:
    """Row/column decomposition used by the multi-GPU path.

    j = j1 + n1*j2, k = k2 + n2*k1:
      X[k2 + n2 k1] = sum_j1 w_n1^(j1 k1) w_n^(j1 k2) sum_j2 w_n2^(j2 k2) x[j1 + n1 j2]
    Returns natural-order X (the distributed path's column-layout output is gathered by tests).
    """
    n = n1 * n2
    assert len(x) == n
    w_n = root_of_unity(p, g, n)
    Y = [[0] * n2 for _ in range(n1)]
    for j1 in range(n1):
        col = ntt_dit([x[j1 + n1 * j2] for j2 in range(n2)], p, g)
        for k2 in range(n2):
            Y[j1][k2] = col[k2] * pow(w_n, j1 * k2, p) % p
    X = [0] * n
    for k2 in range(n2):
        row = ntt_dit([Y[j1][k2] for j1 in range(n1)], p, g)
        for k1 in range(n1):
            X[k2 + n2 * k1] = row[k1]
    return X


def polymul(a: Sequence[int], b: Sequence[int], p: int, g: int) -> List[int]:
    """c = a*b (cyclic of length n = len(a) = len(b)) via forward, pointwise, inverse."""
    A, B = ntt_dit(a, p, g), ntt_dit(b, p, g)
    return intt([u * v % p for u, v in zip(A, B)], p, g)


# ----------------------------------------------------------------------------- limb packing
def to_limbs32(values: Iterable[int], n32: int) -> List[int]:
    """Little-endian 32-bit limbs (cgbn_mem_t<32*n32> layout, cgbn_cuda.h:51-55)."""
    out = []
    m = (1 << 32) - 1
    for v in values:
        for i in range(n32):
            out.append((v >> (32 * i)) & m)
    return out


def from_limbs32(limbs: Sequence[int], n32: int) -> List[int]:
    out = []
    for e in range(len(limbs) // n32):
        v = 0
        for i in range(n32):
            v |= int(limbs[e * n32 + i]) << (32 * i)
        out.append(v)
    return out
