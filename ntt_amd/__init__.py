"""ntt_amd — MI355X-native (gfx950) big-integer NTT.

Hot path: forward/inverse NTT over ~256-bit prime fields (BN254 Fr, BLS12-381 Fr, and the
reference's P = 469762049), natural order in place, behind the C ABI of include/ntt.h
(libntt.so).  See DESIGN.md.
"""
from .fields import FIELDS, BN254_FR, BLS12_381_FR, P469762049  # noqa: F401

__all__ = ["FIELDS", "BN254_FR", "BLS12_381_FR", "P469762049"]
