"""ctypes wrapper of oracle/_ref/libref_{gzkp,ssip}.so — TEST INFRASTRUCTURE ONLY (the checker).

These libraries are the reference's OWN CPU transforms, compiled by ``make -C oracle ref`` from
``/root/reference/src/GZKP-NTT.cu:1-48`` (``NTT``) and ``src/self-sort-in-place.cu:1-128``
(``NTT``, ``NTT_dif``, ``NTT_pro1``, ``NTT_pro2``) where they lie, plus ``oracle/ref_harness.cpp``.
They pin the restatements in ``oracle/ntt_oracle.c`` / ``oracle/ntt_ref.py`` over the reference's
field P = 469762049 (the only field the reference's runnable code has, GZKP-NTT.cu:7).  The
fixtures in ``tests/golden/ref_p469762049.npz`` are their outputs (``tests/golden/make_ref_vectors.py``),
so the pins hold where /root/reference is absent (the GPU box).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")
REF_SRC = os.environ.get("NTT_REFERENCE_ROOT", "/root/reference")
_libs: dict = {}


def build() -> bool:
    """Build oracle/_ref from the reference sources when they are present; True if the libs exist.
    Never fatal: a failed reference compile leaves the checker absent (the committed fixtures in
    tests/golden/ still pin the oracle), it does not fail the product build."""
    if os.path.isdir(os.path.join(REF_SRC, "src")):
        r = subprocess.run(["make", "-C", HERE, "-s", "ref", f"REF={REF_SRC}"], capture_output=True, text=True)
        if r.returncode != 0:
            print(f"oracle/_ref not built (test-only checker): {r.stderr.strip()[-400:]}")
    return available()


def available() -> bool:
    return all(os.path.exists(os.path.join(REF_DIR, f"libref_{k}.so")) for k in ("gzkp", "ssip"))


def _load(kind: str) -> C.CDLL:
    if kind not in _libs:
        lib = C.CDLL(os.path.join(REF_DIR, f"libref_{kind}.so"))
        lib.ref_ntt.restype = C.c_int
        lib.ref_ntt.argtypes = [C.c_void_p, C.c_uint, C.c_longlong, C.c_int]
        lib.ref_modulus.restype = C.c_longlong
        if kind == "ssip":
            lib.ref_ssip_pro.restype = C.c_int
            lib.ref_ssip_pro.argtypes = [C.c_void_p, C.c_uint, C.c_longlong]
            lib.ref_ntt_dif.restype = C.c_int
            lib.ref_ntt_dif.argtypes = [C.c_void_p, C.c_uint, C.c_longlong]
        _libs[kind] = lib
    return _libs[kind]


def _run(fn, x, *args):
    d = np.ascontiguousarray(x, dtype=np.int64).copy()
    log_n = d.size.bit_length() - 1
    assert d.size == 1 << log_n
    assert fn(d.ctypes.data, log_n, *args) == 0
    return d


def ntt(x, omega: int = 3, inverse: bool = False) -> np.ndarray:
    """GZKP-NTT.cu NTT (forward), or the GZKP-NTT.cu:1725-1732 inverse recipe."""
    return _run(_load("gzkp").ref_ntt, x, omega, int(inverse))


def ssip_pro(x, omega: int = 3) -> np.ndarray:
    """self-sort-in-place.cu NTT_pro1 + NTT_pro2."""
    return _run(_load("ssip").ref_ssip_pro, x, omega)


def ntt_dif(x, omega: int = 3) -> np.ndarray:
    """self-sort-in-place.cu NTT_dif (DIF, then the bit-reversal permutation)."""
    return _run(_load("ssip").ref_ntt_dif, x, omega)


def ssip_file_ntt(x, omega: int = 3) -> np.ndarray:
    """self-sort-in-place.cu's own copy of NTT (its main's CPU check)."""
    return _run(_load("ssip").ref_ntt, x, omega, 0)


def modulus() -> int:
    return int(_load("gzkp").ref_modulus())
