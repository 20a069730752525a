"""Field constants (product side).  Kept in sync with ntt_plan.cpp's kFields table."""
from __future__ import annotations

P469762049 = 469762049  # 7 * 2^26 + 1, generator 3 (reference GZKP-NTT.cu:7-8)
BN254_FR = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
BLS12_381_FR = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

FIELDS = {
    0: ("P469762049", P469762049, 3),
    1: ("BN254_FR", BN254_FR, 5),
    2: ("BLS12_381_FR", BLS12_381_FR, 7),
}


def field_params(field_id: int):
    name, p, g = FIELDS[field_id]
    return p, g


def two_adicity(p: int) -> int:
    v, s = p - 1, 0
    while v % 2 == 0:
        v //= 2
        s += 1
    return s
