"""Inputs and the correctness check for tools/mb_limb30.hip (see tools/gen_mb_limb30.py).

    python tools/mb_limb30_check.py prep DIR      # DIR/consts.bin, DIR/xs.bin (BN254 Fr)
    tools/mb_limb30 DIR/consts.bin DIR/xs.bin DIR/rs.bin
    python tools/mb_limb30_check.py verify DIR    # r == x w mod p and 0 <= r < 11 p for every x
"""
import os
import random
import struct
import sys

P = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001  # BN254 Fr
G = 5


def limbs(v, bits, n=9):
    return [(v >> (bits * i)) & ((1 << bits) - 1) for i in range(n)]


def value(ls, bits):
    return sum(x << (bits * i) for i, x in enumerate(ls))


def consts():
    w = pow(G, (P - 1) // 256 * 37, P)  # a radix-256 twiddle
    y = pow(G, 12345, P)
    ws29 = (w << 261) // P
    ws30 = (w << 270) // P
    return w, y, ws29, ws30


def prep(d):
    os.makedirs(d, exist_ok=True)
    w, y, ws29, ws30 = consts()
    words = lambda v, n: [(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)]
    data = words(P, 8) + words(w, 8) + limbs(ws29, 29) + limbs(ws30, 30) + words(y, 8)
    with open(os.path.join(d, "consts.bin"), "wb") as f:
        f.write(struct.pack("<42I", *data))
    rng = random.Random(7)
    xs = []
    # edge cases: zero, max normalised limbs with the largest top limb the pass kernels produce
    # (values < 2^261 after a lazy butterfly), p - 1, multiples of p
    xs.append([0] * 9)
    xs.append([(1 << 30) - 1] * 8 + [(1 << 21) - 1])
    for v in (P - 1, P, 2 * P, 11 * P, (1 << 261) - 1, 64 * P - 1):
        xs.append(limbs(v, 30))
    while len(xs) < 8192:
        v = rng.randrange(1 << 261)
        xs.append(limbs(v, 30))
    with open(os.path.join(d, "xs.bin"), "wb") as f:
        for x in xs:
            f.write(struct.pack("<9I", *x))


def verify(d):
    w, _, _, _ = consts()
    xs = open(os.path.join(d, "xs.bin"), "rb").read()
    rs = open(os.path.join(d, "rs.bin"), "rb").read()
    n = len(xs) // 36
    worst = 0
    for i in range(n):
        x = value(struct.unpack_from("<9I", xs, 36 * i), 30)
        rl = struct.unpack_from("<9I", rs, 36 * i)
        assert all(l < (1 << 30) for l in rl), (i, rl)
        r = value(rl, 30)
        assert r % P == (x * w) % P, (i, hex(x), hex(r))
        assert r < 11 * P, (i, r / P)
        worst = max(worst, r // P)
    print(f'{{"mulc30_checked": {n}, "ok": true, "max_r_over_p": {worst}}}')


if __name__ == "__main__":
    {"prep": prep, "verify": verify}[sys.argv[1]](sys.argv[2])
