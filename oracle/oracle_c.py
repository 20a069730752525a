"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY (the checker, never the product).

Fast C restatement of the reference transform (oracle/ntt_oracle.c) for sizes where the pure-Python
oracle (oracle/ntt_ref.py) is too slow.  Used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
_lib = None


def build() -> str:
    src = os.path.join(HERE, "ntt_oracle.c")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        build()
        lib = C.CDLL(LIB)
        lib.oracle_ntt_u64.restype = C.c_int
        lib.oracle_ntt_u64.argtypes = [C.c_void_p, C.c_uint32, C.c_int64, C.c_int64, C.c_int]
        lib.oracle_ssip_u64.restype = C.c_int
        lib.oracle_ssip_u64.argtypes = [C.c_void_p, C.c_uint32, C.c_int64, C.c_int64]
        lib.oracle_ntt_mp.restype = C.c_int
        lib.oracle_ntt_mp.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int]
        lib.oracle_ntt_mp_par.restype = C.c_int
        lib.oracle_ntt_mp_par.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int,
                                          C.c_int]
        lib.oracle_mul_mp.restype = C.c_int
        lib.oracle_mul_mp.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p]
        lib.oracle_eval_random_mp.restype = C.c_int
        lib.oracle_eval_random_mp.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                              C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int]
        _lib = lib
    return _lib


def _limbs(v: int, L: int) -> np.ndarray:
    return np.array([(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(L)], dtype=np.uint64)


def ntt_u64(x: np.ndarray, p: int, g: int, inverse: bool = False) -> np.ndarray:
    """GZKP-NTT.cu:30-48 over a < 2^31 prime; x: int64 array of length 2^k (copied)."""
    d = np.ascontiguousarray(x, dtype=np.int64).copy()
    log_n = d.size.bit_length() - 1
    rc = load().oracle_ntt_u64(d.ctypes.data, log_n, p, g, int(inverse))
    assert rc == 0
    return d


def ssip_u64(x: np.ndarray, p: int, g: int) -> np.ndarray:
    d = np.ascontiguousarray(x, dtype=np.int64).copy()
    rc = load().oracle_ssip_u64(d.ctypes.data, d.size.bit_length() - 1, p, g)
    assert rc == 0
    return d


def ntt_mp(x: np.ndarray, p: int, g: int, inverse: bool = False) -> np.ndarray:
    """Multi-precision NTT: x is a uint64 array [n, L] of little-endian limbs (copied)."""
    d = np.ascontiguousarray(x, dtype=np.uint64).copy()
    n, L = d.shape
    pl, gl = _limbs(p, L), _limbs(g, L)  # keep the arrays alive across the call
    rc = load().oracle_ntt_mp(d.ctypes.data, n.bit_length() - 1, L, pl.ctypes.data, gl.ctypes.data, int(inverse))
    assert rc == 0
    return d


def ntt_mp_par(x: np.ndarray, p: int, g: int, threads: int, inverse: bool = False) -> np.ndarray:
    """ntt_mp with each stage split over `threads` OpenMP threads (bench.py's multi-core baseline)."""
    d = np.ascontiguousarray(x, dtype=np.uint64).copy()
    n, L = d.shape
    pl, gl = _limbs(p, L), _limbs(g, L)
    rc = load().oracle_ntt_mp_par(d.ctypes.data, n.bit_length() - 1, L, pl.ctypes.data, gl.ctypes.data,
                                  int(inverse), int(threads))
    assert rc == 0
    return d


def mul_mp(a: np.ndarray, b: np.ndarray, p: int) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    c = np.zeros_like(a)
    n, L = a.shape
    pl = _limbs(p, L)
    rc = load().oracle_mul_mp(c.ctypes.data, a.ctypes.data, b.ctypes.data, n, L, pl.ctypes.data)
    assert rc == 0
    return c


RANDOM_SHAPE = {0: (1, 28), 1: (4, 61), 2: (4, 62)}  # field_id -> (random limbs, bits of the top one)


def eval_random(field_id: int, log_n: int, seed: int, ks, L: int, threads: int = 1):
    """X_k of the forward transform of vector B (random_limbs(field_id, 2^log_n, seed, L)) at the
    indices ks, from the definition (oracle_eval_random_mp); returns Python ints."""
    from oracle import ntt_ref as R
    p, g = R.FIELDS[field_id]
    nrand, top = RANDOM_SHAPE[field_id]
    karr = np.ascontiguousarray(np.asarray(ks, dtype=np.uint64))
    out = np.zeros((len(karr), L), dtype=np.uint64)
    pl, gl = _limbs(p, L), _limbs(g, L)
    rc = load().oracle_eval_random_mp(out.ctypes.data, karr.ctypes.data, len(karr), log_n, L, pl.ctypes.data,
                                      gl.ctypes.data, seed, nrand, top, int(threads))
    assert rc == 0
    return limbs_to_ints(out)


def ints_to_limbs(values, L: int) -> np.ndarray:
    out = np.zeros((len(values), L), dtype=np.uint64)
    for j, v in enumerate(values):
        for i in range(L):
            out[j, i] = (int(v) >> (64 * i)) & 0xFFFFFFFFFFFFFFFF
    return out


def limbs_to_ints(arr: np.ndarray):
    res = []
    for row in np.asarray(arr, dtype=np.uint64):
        v = 0
        for i in range(len(row) - 1, -1, -1):
            v = (v << 64) | int(row[i])
        res.append(v)
    return res


def random_limbs(field_id: int, n: int, seed: int, L: int) -> np.ndarray:
    """Vectorised SURVEY §8d vector B (same values as ntt_ref.random_vector), as [n, L] limbs."""
    j = np.arange(n, dtype=np.uint64)
    out = np.zeros((n, L), dtype=np.uint64)
    nrand, top = RANDOM_SHAPE[field_id]
    with np.errstate(over="ignore"):
        for i in range(min(nrand, L)):
            c = (np.uint64(seed) << np.uint64(32)) + np.uint64(4) * j + np.uint64(i)
            z = c + np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            if i == nrand - 1:
                z &= np.uint64((1 << top) - 1)
            out[:, i] = z
    return out
